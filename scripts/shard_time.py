"""Per-shard time of the local part of a sharded run (align + finish: pack,
index, seed, extension, groups, RBH) on one GPU, shard by shard -- the
strong-scaling projection of bench.py --gpus K without the edge exchange and
the (replicated) graph phase.

    python scripts/shard_time.py --config C3 --shards 8
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
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate, CONFIGS
    samples, _ = simulate(**CONFIGS[args.config])
    out = {"config": args.config, "shards": args.shards, "ms": [], "phases": []}
    for r in range(args.shards):
        eng = Engine(device=0, shard_rank=r, shard_count=args.shards)
        for s in samples:
            eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
        eng.upload()
        best = None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.align()
            eng.finish()
            torch.cuda.synchronize()
            dt = 1e3 * (time.perf_counter() - t0)
            best = dt if best is None else min(best, dt)
        out["ms"].append(round(best, 2))
        out["phases"].append({k: round(v, 2) for k, v in eng.timings().items() if k.endswith("_ms")})
        eng.close()
        print(f"shard {r}: {best:.1f} ms", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
