"""A small HDF5 writer and reader for matrix.h5 and the od2 gene matches
tables without PyTables.

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
the classic layout every HDF5 reader since 1.6 understands. Groups of at most 8
children, contiguous datasets (float64, int64, fixed-length strings, and the
compound rows of a PyTables Table), scalar attributes.

The gene matches tables (od2/{s1}--{s2}.h5) are pandas *table* format
(`df.to_hdf(path, key="gene_matches", format="table")`,
gene_matches_tables.py:42-56): `write_frame_table` lays out the same tree --
the frame group with pandas' pickled metadata attributes (protocol 0, as
PyTables stores Python objects), a Table of (index, values_block_k) rows with
one block per pandas dtype block, and a series table per categorical column
(/key/meta/values_block_k/meta). Two things PyTables adds are left out: the
index's search structure (/key/_i_table; `to_hdf(..., index=False)` omits it
too) and chunked storage (the table is contiguous, which PyTables reads).
tests/test_h5_pytables.py reads both kinds of file back with real PyTables +
pandas.
"""
from __future__ import annotations

import os
import pickle
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


def _dt_bitfield(size):
    # class 4 (bit field), version 1; little endian
    return struct.pack("<B3BI", 0x14, 0, 0, 0, size) + struct.pack("<HH", 0, 8 * size)


def _dt_array(dims, base: bytes, base_size: int):
    # class 10 (array), version 2: rank, 3 reserved, sizes, permutation, base type
    n = 1
    for d in dims:
        n *= d
    body = struct.pack("<B3x", len(dims)) + b"".join(struct.pack("<I", d) for d in dims)
    body += b"".join(struct.pack("<I", i) for i in range(len(dims)))
    return struct.pack("<B3BI", 0x2A, 0, 0, 0, n * base_size) + body + base


def _dt_compound(members):
    """members: [(name, offset, member datatype bytes)], total size last:
    class 6, version 2 (array members need it): per member its name (NUL,
    padded to 8), its offset (4 bytes) and its type."""
    *members, size = members
    body = b""
    for name, off, dt in members:
        body += _pad8(name.encode() + b"\0") + struct.pack("<I", off) + dt
    n = len(members)
    return struct.pack("<B3BI", 0x26, n & 0xFF, (n >> 8) & 0xFF, 0, size) + body


def _dt_of_numpy(dt: np.dtype):
    """Datatype bytes of a numpy scalar dtype (as PyTables maps it)."""
    if dt.kind == "b":
        return _dt_bitfield(1)
    if dt.kind in "iu":
        return _dt_int(dt.itemsize, signed=dt.kind == "i")
    if dt.kind == "f" and dt.itemsize == 8:
        return _dt_float64()
    if dt.kind == "S":
        return _dt_string(dt.itemsize, utf8=False)
    raise TypeError(f"unsupported table column dtype {dt}")


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
    def __init__(self, data, attrs=None, typed=None):
        """data: an array; or typed = (datatype bytes, shape, raw bytes)."""
        self.data = data
        self.attrs = dict(attrs or {})
        self.typed = typed

    def write(self, f: _File) -> int:
        dt, shape, raw = self.typed if self.typed is not None else _value(self.data)
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


# ---------------------------------------------------------------- pandas table format
_PT_TABLE = {"CLASS": "TABLE", "TITLE": "", "VERSION": "2.7"}


def _pk(obj) -> bytes:
    """A Python object as PyTables stores it in an attribute: a protocol-0
    pickle (an ASCII string ending in '.')."""
    return pickle.dumps(obj, protocol=0)


def _table_dataset(nrows, columns, attrs):
    """A PyTables Table: columns = [(name, numpy 2-D array (nrows, k) or 1-D
    array)] -> compound rows; 2-D columns are array members of k items."""
    members, off, fields = [], 0, []
    for name, a in columns:
        a = np.asarray(a)
        base = a.dtype
        dt = _dt_of_numpy(base)
        if a.ndim == 2:
            k = a.shape[1]
            dt = _dt_array((k,), dt, base.itemsize)
            fields.append((name, base, (k,), off))
            width = k * base.itemsize
        else:
            fields.append((name, base, (), off))
            width = base.itemsize
        members.append((name, off, dt))
        off += width
    rec = np.zeros(nrows, dtype=np.dtype({"names": [f[0] for f in fields],
                                          "formats": [(f[1], f[2]) if f[2] else f[1] for f in fields],
                                          "offsets": [f[3] for f in fields], "itemsize": off}))
    for name, a in columns:
        rec[name] = a
    return Dataset(None, attrs={**_PT_TABLE, "NROWS": int(nrows), **attrs},
                   typed=(_dt_compound(members + [off]), (nrows,), rec.tobytes()))


def _frame_attrs(pandas_type, table_type, cols, values_cols, data_columns, info):
    return {**_PT_GROUP, "data_columns": _pk(list(data_columns)), "encoding": "UTF-8", "errors": "strict",
            "index_cols": _pk([(0, "index")]), "info": _pk(info), "levels": 1, "nan_rep": "nan",
            "non_index_axes": _pk([(1, list(cols))]), "pandas_type": pandas_type, "pandas_version": "0.15.2",
            "table_type": table_type, "values_cols": _pk(list(values_cols))}


def _strings(values, encoding="UTF-8"):
    enc = [str(v).encode(encoding) for v in values]
    return np.array(enc, dtype=f"S{max([1] + [len(e) for e in enc])}")


def _series_table(values):
    """A Series of strings in table format (a categorical column's categories,
    HDFStore.put(path, Series(categories), format="table"))."""
    v = _strings(values)
    n = len(v)
    info = {1: {"names": [None], "type": "Index"}, "index": {}, "values": {}}
    table = _table_dataset(n, [("index", np.arange(n, dtype=np.int64)), ("values", v)],
                           {"index_kind": "integer", "values_dtype": v.dtype.name, "values_kind": _pk(["values"]),
                            "values_meta": _pk(None)})
    return Group(attrs=_frame_attrs("series_table", "appendable_series", ["values"], ["values"], ["values"], info),
                 children={"table": table})


def frame_table_blocks(df):
    """pandas' blocks of a frame as HDFStore's table writer takes them
    (_create_axes: the consolidated block manager, one values_block each):
    [(column names, values (nrows x k), categories or None, ordered)]."""
    import pandas as pd
    frame = df._consolidate()
    out = []
    for blk in frame._mgr.blocks:
        items = [frame.columns[i] for i in blk.mgr_locs.as_array]
        vals = blk.values
        if isinstance(getattr(vals, "dtype", None), pd.CategoricalDtype):
            out.append((items, np.asarray(vals.codes).reshape(-1, 1), list(vals.categories), bool(vals.ordered)))
            continue
        a = np.asarray(vals)
        if a.ndim == 1:
            a = a.reshape(1, -1)
        a = a.T   # rows x columns of this block
        if a.dtype == object:
            a = _strings(a.ravel()).reshape(a.shape)
        out.append((items, a, None, None))
    return out


def write_frame_table(path, df, key="gene_matches"):
    """Write a DataFrame (integer index; numeric, bool, string and categorical
    columns) the way `df.to_hdf(path, key=key, format="table", index=False)`
    lays it out."""
    import pandas as pd
    if not pd.api.types.is_integer_dtype(df.index.dtype):
        raise TypeError("write_frame_table: the index must be integer")
    nrows = len(df)
    cols = [("index", np.asarray(df.index, dtype=np.int64))]
    tattrs = {"index_kind": "integer"}
    info = {1: {"names": [None], "type": "Index"}, "index": {}}
    names, meta = [], {}
    for k, (items, a, cats, ordered) in enumerate(frame_table_blocks(df)):
        name = f"values_block_{k}"
        names.append(name)
        cols.append((name, a))
        tattrs[f"{name}_kind"] = _pk([str(c) for c in items])
        tattrs[f"{name}_dtype"] = a.dtype.name
        if cats is not None:
            tattrs[f"{name}_meta"] = "category"
            info[name] = {"ordered": ordered}
            meta[name] = Group(attrs=dict(_PT_GROUP), children={"meta": _series_table(cats)})
        else:
            tattrs[f"{name}_meta"] = _pk(None)
            info[name] = {}
    children = {"table": _table_dataset(nrows, cols, tattrs)}
    if meta:
        if len(meta) > 2 * LEAF_K:
            raise ValueError("more categorical blocks than one group node holds")
        children["meta"] = Group(attrs=dict(_PT_GROUP), children=meta)
    frame = Group(attrs=_frame_attrs("frame_table", "appendable_frame", [str(c) for c in df.columns], names, [],
                                     info), children=children)
    write_tree(path, Group(attrs={**_PT_GROUP, "PYTABLES_FORMAT_VERSION": "2.1"}, children={key: frame}))


# ---------------------------------------------------------------- reading tables back
_HDF5_LIBS = ("libhdf5.so.103", "/opt/conda/lib/libhdf5.so.103", "libhdf5.so")


class _Lib:
    """The HDF5 C library through ctypes: enough to read a pandas table-format
    frame (this module's files, or PyTables') where PyTables is absent."""
    _inst = None

    def __init__(self):
        import ctypes
        last = None
        for name in _HDF5_LIBS:
            try:
                L = ctypes.CDLL(name)
                break
            except OSError as e:
                last = e
        else:
            raise ImportError(f"reading .h5 tables needs PyTables or the HDF5 C library ({last})")
        L.H5open()
        hid = ctypes.c_int64
        for fn in ("H5Fopen", "H5Dopen2", "H5Aopen_by_name", "H5Dget_type", "H5Aget_type", "H5Dget_space",
                   "H5Tget_member_type", "H5Tget_super", "H5Oopen"):
            getattr(L, fn).restype = hid
        L.H5Fopen.argtypes = [ctypes.c_char_p, ctypes.c_uint, hid]
        L.H5Dopen2.argtypes = [hid, ctypes.c_char_p, hid]
        L.H5Oopen.argtypes = [hid, ctypes.c_char_p, hid]
        L.H5Dread.argtypes = [hid, hid, hid, hid, hid, ctypes.c_void_p]
        L.H5Aopen_by_name.argtypes = [hid, ctypes.c_char_p, ctypes.c_char_p, hid, hid]
        L.H5Aexists_by_name.argtypes = [hid, ctypes.c_char_p, ctypes.c_char_p, hid]
        L.H5Lexists.argtypes = [hid, ctypes.c_char_p, hid]
        L.H5Aread.argtypes = [hid, hid, ctypes.c_void_p]
        L.H5Tget_size.restype = ctypes.c_size_t
        L.H5Tget_member_offset.restype = ctypes.c_size_t
        L.H5Tget_member_name.restype = ctypes.c_void_p
        L.H5Tget_member_name.argtypes = [hid, ctypes.c_uint]
        L.H5Tget_member_offset.argtypes = [hid, ctypes.c_uint]
        L.H5Tget_member_type.argtypes = [hid, ctypes.c_uint]
        L.H5Tget_array_dims2.argtypes = [hid, ctypes.c_void_p]
        L.H5free_memory.argtypes = [ctypes.c_void_p]
        for fn in ("H5Dget_type", "H5Aget_type", "H5Tget_size", "H5Dget_space", "H5Fclose", "H5Dclose",
                   "H5Aclose", "H5Tclose", "H5Sclose", "H5Oclose", "H5Sget_simple_extent_ndims",
                   "H5Tget_class", "H5Tget_nmembers", "H5Tget_super", "H5Tget_sign", "H5Tget_array_ndims"):
            getattr(L, fn).argtypes = [hid]
        L.H5Sget_simple_extent_dims.argtypes = [hid, ctypes.c_void_p, ctypes.c_void_p]
        self.L, self.ct = L, ctypes

    @classmethod
    def get(cls):
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def np_dtype(self, t):
        """numpy dtype of an HDF5 atomic/array type (no compound)."""
        L = self.L
        cls, size = L.H5Tget_class(t), L.H5Tget_size(t)
        if cls == 0:    # integer
            return np.dtype(f"<{'i' if L.H5Tget_sign(t) == 1 else 'u'}{size}")
        if cls == 1:    # float
            return np.dtype(f"<f{size}")
        if cls == 3:    # string
            return np.dtype(f"S{size}")
        if cls == 4:    # bit field (PyTables' bool)
            return np.dtype(bool)
        if cls == 10:   # array
            nd = L.H5Tget_array_ndims(t)
            dims = (self.ct.c_uint64 * nd)()
            L.H5Tget_array_dims2(t, dims)
            base = L.H5Tget_super(t)
            try:
                return np.dtype((self.np_dtype(base), tuple(dims[i] for i in range(nd))))
            finally:
                L.H5Tclose(base)
        raise TypeError(f"unsupported HDF5 type class {cls}")

    def table(self, f, path):
        """A Table dataset -> numpy structured array (the file's own layout)."""
        L, ct = self.L, self.ct
        d = L.H5Dopen2(f, path.encode(), 0)
        if d < 0:
            raise KeyError(path)
        t = L.H5Dget_type(d)
        names, formats, offsets = [], [], []
        for i in range(L.H5Tget_nmembers(t)):
            p = L.H5Tget_member_name(t, i)
            names.append(ct.string_at(p).decode())
            L.H5free_memory(p)
            mt = L.H5Tget_member_type(t, i)
            formats.append(self.np_dtype(mt))
            L.H5Tclose(mt)
            offsets.append(L.H5Tget_member_offset(t, i))
        dt = np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": L.H5Tget_size(t)})
        sp = L.H5Dget_space(d)
        n = (ct.c_uint64 * 1)()
        L.H5Sget_simple_extent_dims(sp, n, None)
        out = np.zeros(n[0], dtype=dt)
        if n[0] and L.H5Dread(d, t, 0, 0, 0, out.ctypes.data) < 0:
            raise OSError(f"H5Dread of {path} failed")
        for h, close in ((sp, L.H5Sclose), (t, L.H5Tclose), (d, L.H5Dclose)):
            close(h)
        return out

    def attr(self, f, obj, name):
        """A string attribute (pickled ones unpickled), an integer, or None."""
        L, ct = self.L, self.ct
        if L.H5Aexists_by_name(f, obj.encode(), name.encode(), 0) <= 0:
            return None
        a = L.H5Aopen_by_name(f, obj.encode(), name.encode(), 0, 0)
        t = L.H5Aget_type(a)
        cls, size = L.H5Tget_class(t), L.H5Tget_size(t)
        buf = ct.create_string_buffer(max(size, 1))
        L.H5Aread(a, t, buf)
        L.H5Tclose(t)
        L.H5Aclose(a)
        if cls == 0:
            return int(np.frombuffer(buf.raw[:size], dtype=f"<i{size}")[0])
        raw = buf.raw[:size].rstrip(b"\0")
        if raw.endswith(b"."):
            try:
                return pickle.loads(raw)
            except Exception:
                pass
        return raw.decode()


def read_frame_table(path, key="gene_matches"):
    """A pandas table-format frame (write_frame_table's, or PyTables') back
    as a DataFrame, through the HDF5 C library -- for read_table where
    PyTables is absent."""
    import pandas as pd
    H = _Lib.get()
    f = H.L.H5Fopen(os.fspath(path).encode(), 0, 0)
    if f < 0:
        raise OSError(f"cannot open {path}")
    try:
        g = "/" + key
        if H.L.H5Lexists(f, g.encode(), 0) <= 0:
            raise KeyError(f"No object named {key} in the file")
        cols = H.attr(f, g, "non_index_axes")[0][1]
        rec = H.table(f, g + "/table")
        data = {}
        for name in H.attr(f, g, "values_cols"):
            items = H.attr(f, g + "/table", f"{name}_kind")
            meta = H.attr(f, g + "/table", f"{name}_meta")
            dtype = H.attr(f, g + "/table", f"{name}_dtype")
            block = rec[name].reshape(len(rec), len(items))
            cats = None
            if meta == "category":
                cats = [v.decode() for v in H.table(f, f"{g}/meta/{name}/meta/table")["values"]]
                ordered = bool(H.attr(f, g, "info").get(name, {}).get("ordered", False))
            for j, c in enumerate(items):
                v = block[:, j]
                if cats is not None:
                    data[c] = pd.Categorical.from_codes(v.astype(np.int64), categories=cats, ordered=ordered)
                elif str(dtype).startswith("bytes"):
                    data[c] = np.array([x.decode() for x in v], dtype=object)
                else:
                    data[c] = v.astype(np.dtype(dtype), copy=False)
        index = pd.Index(rec["index"].astype(np.int64))
        return pd.DataFrame({c: data[c] for c in cols}, index=index)
    finally:
        H.L.H5Fclose(f)
