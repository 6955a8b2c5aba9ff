"""One summary line of a bench JSON (A/B runs through scripts/gpu.sh)."""
import json
import sys

d = json.load(open(sys.argv[1]))
p = d["phases_ms"]
print(sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] else "default", d["value"], d["ms_per_step"],
      *(f"{k} {p.get(k)}" for k in ("pack_ms", "dust_ms", "index_ms", "seed_kernel_ms", "align_kernel_ms", "rbh_ms")))
