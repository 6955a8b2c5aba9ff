"""Where a step's wall time goes, from a rocprofv3 --kernel-trace --hip-trace
run of `bench.py --shard R/S` (1 warmup + 1 step): the last step is the last
`tiles` pack_fwd launches on. Prints JSON: the step's span, the time some
kernel was running (union of kernel intervals), the idle gaps between kernels
(count, total, the largest with the kernels around them and the HIP calls
inside), per-kernel totals, and per-HIP-function totals inside the step.

    python scripts/trace_gaps.py PROFILE_DIR TILES [OUT.json]
"""
import collections
import csv
import glob
import json
import sys


def load(d, pat):
    fs = sorted(glob.glob(f"{d}/**/*{pat}", recursive=True))
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main():
    d, tiles = sys.argv[1], int(sys.argv[2])
    ks = sorted(load(d, "kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    api = load(d, "hip_api_trace.csv")
    packs = [i for i, r in enumerate(ks) if "pack_fwd" in r["Kernel_Name"]]
    i0 = packs[-tiles] if len(packs) >= tiles else 0
    ks = ks[i0:]
    t0 = int(ks[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in ks)
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:60])
          for r in ks]
    busy, gaps, cur_s, cur_e, prev = 0, [], iv[0][0], iv[0][1], iv[0][2]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, s, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n if e >= cur_e else prev
    busy += cur_e - cur_s
    tot = collections.Counter()
    for s, e, n in iv:
        tot[n] += e - s
    calls = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api
             if int(r["End_Timestamp"]) >= t0 and int(r["Start_Timestamp"]) <= t1]
    ftot, fcnt = collections.Counter(), collections.Counter()
    for s, e, f in calls:
        ftot[f] += e - s
        fcnt[f] += 1
    big = sorted(gaps, reverse=True)[:25]
    out = {
        "step_span_ms": round((t1 - t0) / 1e6, 1),
        "kernel_busy_ms": round(busy / 1e6, 1),
        "busy_frac": round(busy / max(1, t1 - t0), 3),
        "gaps": {"n": len(gaps), "total_ms": round(sum(g[0] for g in gaps) / 1e6, 1),
                 "over_1ms": sum(1 for g in gaps if g[0] > 1e6),
                 "over_1ms_total_ms": round(sum(g[0] for g in gaps if g[0] > 1e6) / 1e6, 1)},
        "largest_gaps": [{
            "ms": round(g[0] / 1e6, 2), "at_ms": round((g[1] - t0) / 1e6, 1), "after": g[3], "before": g[4],
            "hip_calls": [f"{f} {(e - s) / 1e6:.2f}ms" for s, e, f in calls
                          if s < g[2] and e > g[1] and (e - s) > 2e5][:8]} for g in big],
        "kernels_ms": {k: round(v / 1e6, 1) for k, v in tot.most_common(25)},
        "hip_api_ms": {f: [round(v / 1e6, 1), fcnt[f]] for f, v in ftot.most_common(25)},
    }
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s)


if __name__ == "__main__":
    main()
