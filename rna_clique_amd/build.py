"""Build librcgpu.so in-tree with hipcc for gfx950 (no JIT cache, no pip)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "librcgpu.so")
SOURCES = ["kernels.hip", "sort.hip", "align.hip", "dust.hip", "engine.hip", "fasta.cpp", "graph_pickle.cpp",
           "od2_tables.cpp"]
HEADERS = ["device.h", os.path.join("..", "..", "include", "rcgpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread",
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(out, defines=(), verbose=False):
    """One object per source, compiled in parallel (each source is
    self-contained: kernels are launched from their own file), then linked."""
    from concurrent.futures import ThreadPoolExecutor
    import tempfile
    extra = os.environ.get("RC_EXTRA_FLAGS", "").split()
    cflags = [f for f in FLAGS if f != "-shared"] + list(defines) + extra
    with tempfile.TemporaryDirectory(prefix="rcgpu_") as tmp:
        objs = [os.path.join(tmp, s + ".o") for s in SOURCES]

        def one(i):
            cmd = [HIPCC, *cflags, "-c", "-o", objs[i], SOURCES[i]]
            return cmd, subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)

        with ThreadPoolExecutor(min(len(SOURCES), os.cpu_count() or 4)) as ex:
            results = list(ex.map(one, range(len(SOURCES))))
        for cmd, res in results:
            if res.returncode != 0:
                raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{res.stderr[-8000:]}")
            if verbose and res.stderr:
                print(res.stderr)
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-pthread", "-o", out + ".tmp", *objs]
        res = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{res.stderr[-8000:]}")
    os.replace(out + ".tmp", out)
    return out


def build_native(force=False, verbose=False):
    """Compile the HIP engine into rna_clique_amd/librcgpu.so."""
    if not force and not _stale():
        return OUT
    return _compile(OUT, verbose=verbose)


def build_timing():
    """The same library with the row-extension cycle counters compiled in
    (RC_ROW_TIMING), as librcgpu_timing.so, for profiling runs (RC_LIB=...)."""
    return _compile(os.path.join(HERE, "librcgpu_timing.so"), defines=("-DRC_ROW_TIMING",))
