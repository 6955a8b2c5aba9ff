"""PyTables + pandas as a checker of this package's HDF5 writers.

TEST INFRASTRUCTURE ONLY. The image's main interpreter has no PyTables, but
/opt/conda carries a Python 3.9 with PyTables 3.6.1, h5py and pandas 2.3.
PyTables 3.6 predates numpy 1.24, so the removed numpy aliases it imports are
restored first (and pandas' minimum-version gate is told 3.8), which is
enough for `to_hdf` / `read_hdf` round trips. Run by tests/test_h5_pytables.py
as a subprocess:

    python3.9 pytables_ref.py read  PATH KEY OUT.json   # read_hdf -> JSON
    python3.9 pytables_ref.py write IN.json PATH KEY FORMAT   # to_hdf from JSON
"""
import json
import sys

import numpy as np

np.typeDict = np.sctypeDict
for _n, _t in (("bool", bool), ("int", int), ("float", float), ("object", object), ("str", str),
               ("complex", complex)):
    if not hasattr(np, _n):
        setattr(np, _n, _t)
import tables  # noqa: E402

tables.__version__ = "3.8.0"
import pandas as pd  # noqa: E402


def frame_to_json(df):
    cols = {}
    for c in df.columns:
        s = df[c]
        if isinstance(s.dtype, pd.CategoricalDtype):
            cols[str(c)] = {"dtype": "category", "categories": [str(x) for x in s.cat.categories],
                            "values": [str(x) for x in s.astype(object)]}
        elif s.dtype == object:
            cols[str(c)] = {"dtype": "object", "values": [str(x) for x in s]}
        else:
            cols[str(c)] = {"dtype": str(s.dtype), "values": s.to_numpy().tolist()}
    return {"index": [x if isinstance(x, (int, float)) else str(x) for x in df.index.tolist()],
            "index_dtype": str(df.index.dtype), "columns": [str(c) for c in df.columns], "data": cols}


def json_to_frame(d):
    data = {}
    for c in d["columns"]:
        col = d["data"][c]
        if col["dtype"] == "category":
            data[c] = pd.Categorical(col["values"], categories=col["categories"])
        elif col["dtype"] == "object":
            data[c] = pd.Series(col["values"], dtype=object).to_numpy()
        else:
            data[c] = np.asarray(col["values"], dtype=col["dtype"])
    idx = pd.Index(np.asarray(d["index"], dtype=d.get("index_dtype", "int64")))
    return pd.DataFrame(data, index=idx, columns=d["columns"])


def main():
    cmd = sys.argv[1]
    if cmd == "read":
        df = pd.read_hdf(sys.argv[2], key=sys.argv[3])
        with open(sys.argv[4], "w") as f:
            json.dump(frame_to_json(df), f)
    elif cmd == "write":
        with open(sys.argv[2]) as f:
            df = json_to_frame(json.load(f))
        df.to_hdf(sys.argv[3], key=sys.argv[4], format=sys.argv[5])
    else:
        raise SystemExit(f"unknown command {cmd}")


if __name__ == "__main__":
    main()
