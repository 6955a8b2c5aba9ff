"""Summarise rocprofv3 PMC passes (scripts/gpu_pmc.sh) per kernel.

Usage: python scripts/pmc_summary.py gpurun_out/pmc_C3 profiles/<round>/C3_pmc.json [commit]
       [kernel_stats.csv runs]

With a `rocprofv3 --kernel-trace --stats` CSV of the same sources and the
number of bench steps it covers (warmup included), the issue entry also
carries the row kernel's own time per step, so bench.py can price its VALU
count against that kernel alone rather than against every extension kernel.

The summary is stamped with bench.src_hash() of the sources in this tree
(run it on the tree the profile was measured on); bench.py reports PMC
traffic only from a summary whose stamp matches its own sources.

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


# VALU issue peak, wave instructions / ns: 256 CUs x 4 SIMDs x 2.4 GHz, a wave64
# VALU instruction occupying a 32-lane SIMD for 2 clocks (MI355X_MICROARCH.md)
VALU_PEAK_G = 256 * 4 * 2.4 / 2


def _ext_steps(src):
    """Greedy row steps of the profiled bench step (bench JSON in the pass logs)."""
    for f in sorted(glob.glob(src.rstrip("/") + "_p*.log")):
        for line in open(f):
            if line.startswith("{"):
                try:
                    return json.loads(line)["phases_ms"]["ext_steps"]
                except (ValueError, KeyError):
                    pass
    return None


def _rows_ms(stats, runs):
    """extend_rows_kernel<..., 32, ...> (the sliding rows) ms per step from a
    kernel-stats CSV covering `runs` steps."""
    tot = 0.0
    for r in csv.DictReader(open(stats)):
        if "extend_rows_kernel" in r["Name"] and ", 32," in r["Name"]:
            tot += float(r["TotalDurationNs"])
    return round(tot / 1e6 / runs, 3) if tot else None


def main(src, dst, commit=None, stats=None, runs=None):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import src_hash
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(os.path.join(src, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {"source": src, "commit": commit, "src_hash": src_hash(),
           "note": "per bench step (1 step); FETCH_SIZE/WRITE_SIZE KiB; FETCH_SIZE doubled "
                   "for HBM bytes (MI355X_MICROARCH.md, HBM)",
           "kernels": {k: dict(v) for k, v in agg.items()}}
    tb = 0.0
    for k in ("seed_kernel", "extend_rows_kernel", "extend_kernel", "ext_finish_kernel", "first_finish_kernel"):
        v = agg.get(k, {})
        tb += 2 * 1024 * v.get("FETCH_SIZE", 0.0) + 1024 * v.get("WRITE_SIZE", 0.0)
    out["traffic_bytes_seed_extend"] = int(tb)
    ext = agg.get("extend_rows_kernel", {})
    if "SQ_INSTS_VALU" in ext:
        steps = _ext_steps(src)
        wi = ext.get("SQ_INSTS_VALU", 0.0) + ext.get("SQ_INSTS_SALU", 0.0)
        out["issue"] = {"kernel": "extend_rows_kernel", "wave_instr": wi, "valu_peak_g_per_s": VALU_PEAK_G,
                        "valu": ext.get("SQ_INSTS_VALU"), "salu": ext.get("SQ_INSTS_SALU"),
                        "valu_per_wave_step": round(ext["SQ_INSTS_VALU"] / (steps / 2), 1) if steps else None}
        if stats:
            out["issue"]["kernel_ms"] = _rows_ms(stats, int(runs))
            out["issue"]["kernel_ms_source"] = stats
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: out["kernels"].get(k) for k in ("seed_kernel", "extend_rows_kernel")}, indent=1))
    print("traffic_bytes_seed_extend", out["traffic_bytes_seed_extend"])


if __name__ == "__main__":
    main(*sys.argv[1:])
