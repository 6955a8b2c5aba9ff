"""Wall-clock of the engine's one-time phases on a fresh engine (the e2e
path's engine_s): create, add_sample x N, upload, first run, second run.

    python scripts/engine_phases.py --config C3
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    args = ap.parse_args()
    import torch
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate, CONFIGS
    samples, _ = simulate(**CONFIGS[args.config])
    out = {}
    t = time.perf_counter()

    def lap(k):
        nonlocal t
        torch.cuda.synchronize()
        now = time.perf_counter()
        out[k] = round(now - t, 3)
        t = now
    torch.cuda.init()
    lap("cuda_init")
    eng = Engine(device=0)
    lap("create")
    for s in samples:
        eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    lap("add_samples")
    eng.upload()
    lap("upload")
    eng.run()
    lap("run1")
    out["run1_phases_ms"] = {k: round(v, 1) for k, v in eng.timings().items() if k.endswith("_ms")}
    eng.run()
    lap("run2")
    eng.distance()
    lap("distance")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
