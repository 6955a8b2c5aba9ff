"""One step's kernel timeline from a rocprofv3 --kernel-trace CSV: every
kernel of the last step (from its last pack_fwd_kernel) over 100 us or after
an idle gap over 20 us, with its start, duration, the idle gap before it and
its queue, then the span and the total idle time.

  python scripts/trace_step.py gpurun_out/<tag>/C3_stats/run_kernel_trace.csv
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "pack_fwd_kernel" in r["Kernel_Name"]][-1]
t0 = int(rows[st]["Start_Timestamp"])
busy_end, gaps = t0, 0
for r in rows[st:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = s - busy_end
    gaps += max(gap, 0)
    d = (e - s) / 1e3
    if d > 100 or gap > 20000:
        print(f"{(s - t0) / 1e6:8.3f} ms  dur {d:9.1f} us  gap {max(gap, 0) / 1e3:7.1f}  q{r['Queue_Id']} "
              f"{r['Kernel_Name'][:80]}")
    busy_end = max(busy_end, e)
print(f"span {(busy_end - t0) / 1e6:.3f} ms; idle gaps {gaps / 1e6:.3f} ms")
