"""Summarise rocprofv3 PMC passes (scripts/gpu_pmc.sh) per kernel.

Usage: python scripts/pmc_summary.py gpurun_out/pmc_C3 profiles/<round>/C3_pmc.json [commit]

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so
it is doubled (uncalibrated for other access widths; see that section).
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    for k in ("seed_kernel", "extend_rows_kernel", "ext_finish_kernel", "first_finish_kernel", "extend_kernel", "rbh_kernel", "kmer_fill", "radix_sort", "pack_fwd",
              "pack_rc", "bucket_fill", "mirror_scatter", "mirror_sort", "group_count", "group_write",
              "cc_hook", "cc_count", "pair_sums"):
        if k in name:
            return k
    if "onesweep" in name or "radix" in name.lower():
        return "radix_sort"
    return name.split("(")[0][-40:]


def main(src, dst, commit=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {"source": src, "commit": commit, "note": "per bench step (1 step, C3); FETCH_SIZE/WRITE_SIZE KiB",
           "kernels": {k: dict(v) for k, v in agg.items()}}
    tb = 0.0
    for k in ("seed_kernel", "extend_rows_kernel", "extend_kernel", "ext_finish_kernel"):
        v = agg.get(k, {})
        tb += 2 * 1024 * v.get("FETCH_SIZE", 0.0) + 1024 * v.get("WRITE_SIZE", 0.0)
    out["traffic_bytes_seed_extend"] = int(tb)
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: out["kernels"].get(k) for k in ("seed_kernel", "extend_rows_kernel")}, indent=1))
    print("traffic_bytes_seed_extend", out["traffic_bytes_seed_extend"])


if __name__ == "__main__":
    main(*sys.argv[1:])
