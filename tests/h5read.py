"""Read HDF5 files back through the real HDF5 C library (ctypes), to check
rna_clique_amd.h5's writer. Test helper only; skipped where libhdf5 is absent."""
import ctypes

import numpy as np

LIBHDF5 = "/opt/conda/lib/libhdf5.so.103"


class H5:
    """Just enough of the HDF5 C API (via ctypes) to read a file back."""

    def __init__(self):
        L = ctypes.CDLL(LIBHDF5)
        L.H5open()
        hid = ctypes.c_int64
        for fn in ["H5Fopen", "H5Dopen2", "H5Aopen_by_name", "H5Dget_type", "H5Aget_type",
                   "H5Gopen2", "H5Dget_space"]:
            getattr(L, fn).restype = hid
        L.H5Tget_size.restype = ctypes.c_size_t
        L.H5Fopen.argtypes = [ctypes.c_char_p, ctypes.c_uint, hid]
        L.H5Dopen2.argtypes = [hid, ctypes.c_char_p, hid]
        L.H5Gopen2.argtypes = [hid, ctypes.c_char_p, hid]
        L.H5Dread.argtypes = [hid, hid, hid, hid, hid, ctypes.c_void_p]
        L.H5Aopen_by_name.argtypes = [hid, ctypes.c_char_p, ctypes.c_char_p, hid, hid]
        L.H5Aread.argtypes = [hid, hid, ctypes.c_void_p]
        for fn in ["H5Dget_type", "H5Aget_type", "H5Tget_size", "H5Dget_space", "H5Fclose",
                   "H5Sget_simple_extent_ndims"]:
            getattr(L, fn).argtypes = [hid]
        L.H5Sget_simple_extent_dims.argtypes = [hid, ctypes.c_void_p, ctypes.c_void_p]
        L.H5Gget_info.argtypes = [hid, ctypes.c_void_p]
        self.L, self.hid = L, hid
        self.dbl = hid.in_dll(L, "H5T_NATIVE_DOUBLE_g").value

    def open(self, path):
        f = self.L.H5Fopen(str(path).encode(), 0, 0)
        assert f > 0
        return f

    def dims(self, d):
        sp = self.L.H5Dget_space(d)
        nd = self.L.H5Sget_simple_extent_ndims(sp)
        dims = (ctypes.c_uint64 * max(nd, 1))()
        self.L.H5Sget_simple_extent_dims(sp, dims, None)
        return tuple(dims[i] for i in range(nd))

    def doubles(self, f, name):
        d = self.L.H5Dopen2(f, name.encode(), 0)
        assert d > 0
        out = np.zeros(self.dims(d))
        assert self.L.H5Dread(d, self.dbl, 0, 0, 0, out.ctypes.data) >= 0
        return out

    def strings(self, f, name):
        d = self.L.H5Dopen2(f, name.encode(), 0)
        t = self.L.H5Dget_type(d)
        sz = self.L.H5Tget_size(t)
        n = self.dims(d)[0]
        b = ctypes.create_string_buffer(sz * n)
        assert self.L.H5Dread(d, t, 0, 0, 0, b) >= 0
        return [b.raw[i * sz:(i + 1) * sz].rstrip(b"\0").decode() for i in range(n)]

    def attr(self, f, obj, name):
        a = self.L.H5Aopen_by_name(f, obj.encode(), name.encode(), 0, 0)
        assert a > 0, (obj, name)
        t = self.L.H5Aget_type(a)
        sz = self.L.H5Tget_size(t)
        b = ctypes.create_string_buffer(max(sz, 1))
        assert self.L.H5Aread(a, t, b) >= 0
        return b.raw

    def n_links(self, f, group):
        g = self.L.H5Gopen2(f, group.encode(), 0)
        info = (ctypes.c_uint64 * 4)()
        assert self.L.H5Gget_info(g, info) >= 0
        return int(info[1])   # H5G_info_t: storage_type (enum, padded), nlinks, ...
