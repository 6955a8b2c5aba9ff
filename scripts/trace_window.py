"""Print the kernels of the last step's index phase from a rocprofv3
kernel-trace CSV: start / end relative to the step's k-mer fill, queue, name.
Usage: python scripts/trace_window.py TRACE.csv [FIRST_KERNEL_SUBSTRING] [COUNT]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "kmer_fill_hist"
count = int(sys.argv[3]) if len(sys.argv) > 3 else 20
i0 = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]][-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[max(i0 - 2, 0):i0 + count]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{s:9.3f} {e:9.3f} {e - s:8.3f}  q{r['Queue_Id']}  {r['Kernel_Name'][:72]}")
