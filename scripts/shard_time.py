"""Per-shard time of the local part of a sharded run (align + finish: pack,
index, seed, extension, groups, RBH) on one GPU, shard by shard -- the
strong-scaling projection of bench.py --gpus K without the edge exchange and
the (replicated) graph phase.

    python scripts/shard_time.py --config C3 --shards 8 [--share-dust]

--share-dust: the DUST masks are made once per sample across the ranks
(distributed.exchange_dust): a rank's timed work is its own samples' masks
(rc_dust_masks, into a device buffer) plus its alignment with every mask
given (rc_set_dust_masks, device to device); the other ranks' masks are made
untimed beforehand, and the all-gather is modelled (`exchange_model_ms`: the
gathered bytes at 100 GB/s).
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
    ap.add_argument("--share-dust", action="store_true")
    args = ap.parse_args()
    import numpy as np
    import torch
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate, CONFIGS
    samples, _ = simulate(**CONFIGS[args.config])
    out = {"config": args.config, "shards": args.shards, "share_dust": args.share_dust, "ms": [], "phases": []}
    bases = [len(s.seq) for s in samples]
    owner = distributed.dust_owners(bases, args.shards)
    if args.share_dust:
        out["exchange_model_ms"] = round(sum(bases) / 8 / 100e9 * 1e3, 2)
        out["dust_owned_gbp"] = [round(sum(b for b, o in zip(bases, owner) if o == r) / 1e9, 3)
                                 for r in range(args.shards)]
    for r in range(args.shards):
        eng = Engine(device=0, shard_rank=r, shard_count=args.shards)
        for s in samples:
            eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
        eng.upload()
        if args.share_dust:
            need = sorted(distributed.needed_samples(bases, args.shards, r))
            mine = [s for s in need if owner[s] == r]
            others = [s for s in need if owner[s] != r]
            # the other ranks' share, made untimed (on the device, as after the all-gather)
            other_w = torch.from_numpy(eng.dust_masks(others).view(np.int64)).cuda()
            n_own = sum((bases[s] + 63) // 64 for s in mine)
            allw = torch.empty(n_own + other_w.numel(), dtype=torch.int64, device="cuda")
            allw[n_own:] = other_w
        best = None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if args.share_dust:
                eng.dust_masks(mine, allw[:n_own])    # this rank's masks, device to device
                eng.set_dust_masks(mine + others, allw)
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
