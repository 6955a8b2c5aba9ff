"""Timeline of one step's index phase from a rocprofv3 kernel trace (csv):
every kernel from the first pack to the first seed kernel, with its queue,
start offset and duration (ms). Usage: python scripts/trace_index.py TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
packs = [i for i, r in enumerate(rows) if "pack_fwd" in r["Kernel_Name"]]
i0 = packs[-1] if packs else 0
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} ms q{r["Queue_Id"]} {r["Kernel_Name"][:70]}')
    if "seed_kernel" in r["Kernel_Name"]:
        break
