"""Per-launch timeline of the last bench step in a rocprofv3 kernel trace
(launches over 50 us), and the per-kernel totals of that step."""
import collections
import csv
import glob
import sys

f = sorted(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last step starts at the last pack_fwd launch
starts = [i for i, r in enumerate(rows) if "pack_fwd" in r["Kernel_Name"]]
rows = rows[starts[-1]:] if starts else rows
t0 = int(rows[0]["Start_Timestamp"])
tot = collections.Counter()
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    tot[name] += e - s
    if e - s >= 50000:
        print(f"{(s - t0) / 1e6:9.2f} {(e - s) / 1e6:8.3f} ms  {name}")
print(f"step span {(int(rows[-1]['End_Timestamp']) - t0) / 1e6:.2f} ms")
for k, v in tot.most_common(20):
    print(f"{v / 1e6:9.3f} ms  {k}")
