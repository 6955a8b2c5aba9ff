"""HBM residency of one C5 rank through the real sharded sequence, on one GPU.

A rank of the 8-GPU C5 job (BASELINE configs[4]) holds, one after another in
ONE engine: the DUST masks of all 128 samples (the all-gather's result, 1 bit
per base), its alignment working set (tiles, index, seeds, candidates), its
HSP store / rows / edges, then the edge exchange's receive buffer (8 ranks x
the largest count x 20 B) and the imported records with the graph arrays
(distributed.sharded_run). This script runs that sequence for one rank over a
world-1 RCCL group, emulating the seven other ranks' buffers at full size:
* the DUST all-gather buffer holds every sample's mask slot (the rank's own
  masks from rc_dust_masks, zeros for the samples it does not hold -- their
  masks are never read by this rank), gathered in place over RCCL;
* the edge receive buffer has 8 slots of the rank's own record count, the
  rank's records exported into its slot, gathered in place over RCCL, then
  copied into the other seven slots (valid records; the graph phase runs over
  8x the rank's edges, the size of the real exchange).
Device memory is sampled every 2 ms by a thread (hipMemGetInfo: engine and
torch allocations together); the engine's own peak (rc_timing.dev_peak_bytes)
and torch's allocator peaks are reported beside it.

    python scripts/c5_residency.py [--config C5s] [--rank R] [--shards 8] [--trim auto|yes|no]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Sampler:
    def __init__(self, torch):
        self.torch, self.stop, self.peak, self.total = torch, threading.Event(), 0, 0
        self.marks = []
        self.t = threading.Thread(target=self._run, daemon=True)

    def used(self):
        free, total = self.torch.cuda.mem_get_info(0)
        self.total = total
        return total - free

    def _run(self):
        t0, last = time.time(), time.time()
        while not self.stop.wait(0.002):
            self.peak = max(self.peak, self.used())
            if time.time() - last > 30:
                print(f"  ... {time.time() - t0:.0f} s, device peak so far {self.peak / 1e9:.1f} GB", flush=True)
                last = time.time()

    def mark(self, what):
        u = self.used()
        self.peak = max(self.peak, u)
        self.marks.append({"after": what, "device_used_gb": round(u / 1e9, 2),
                           "peak_so_far_gb": round(self.peak / 1e9, 2)})
        print(json.dumps(self.marks[-1]), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5s")
    ap.add_argument("--rank", type=int, default=-1, help="default: the rank with the largest modelled footprint")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--trim", default="auto", choices=["auto", "yes", "no"])
    ap.add_argument("--out", default="gpurun_out/c5_residency.json")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    torch.cuda.init()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    import numpy as np
    from bench import shard_samples
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import CONFIGS, simulate
    S = args.shards
    cfg = dict(CONFIGS[args.config])
    meta, _ = simulate(only=[], **cfg)
    bases = [int(s.tx_offsets[-1]) for s in meta]
    genes = [len(np.unique(s.gene)) for s in meta]
    model = distributed.hbm_footprint(bases, genes, S)
    R = args.rank if args.rank >= 0 else int(np.argmax(model))
    del meta
    print(f"rank {R} of {S}: modelled {model[R] / 1e9:.1f} GB", flush=True)
    samples, need, _ = shard_samples(args.config, S, R)
    smp = Sampler(torch)
    smp.t.start()
    smp.mark("start")
    eng = Engine(device=0, shard_rank=R, shard_count=S)
    for i, s in enumerate(samples):
        eng.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
    del samples
    eng.upload()
    smp.mark("upload")
    t = {}
    # 1. DUST masks: every sample's slot, this rank's own masks in theirs
    t0 = time.perf_counter()
    mine = sorted(need)
    words = [(bases[s] + 63) // 64 for s in range(len(bases))]
    off = np.concatenate([[0], np.cumsum(words)]).astype(np.int64)
    allm = torch.zeros(int(off[-1]), dtype=torch.int64, device="cuda")
    own = torch.empty(sum(words[s] for s in mine), dtype=torch.int64, device="cuda")
    eng.dust_masks(mine, own)
    o = 0
    for s in mine:
        allm[off[s]:off[s + 1]].copy_(own[o:o + words[s]])
        o += words[s]
    del own
    dist.all_gather_into_tensor(allm, allm)   # world 1, in place: the RCCL call of the real exchange
    torch.cuda.synchronize()
    eng.set_dust_masks(list(range(len(bases))), allm)
    del allm
    t["dust_exchange_s"] = round(time.perf_counter() - t0, 3)
    smp.mark("dust masks set")
    # 2. alignment + RBH
    t0 = time.perf_counter()
    eng.align()
    eng.finish()
    t["align_finish_s"] = round(time.perf_counter() - t0, 3)
    tm = eng.timings()
    smp.mark("align + finish")
    # 3. the edge exchange of exchange_edges, 8 slots
    t0 = time.perf_counter()
    rs = Engine.edge_record_size()
    n = eng.local_edge_count()
    counts = [n] * S
    mx = n
    free, _ = torch.cuda.mem_get_info()
    need_b = (S * mx + sum(counts)) * rs
    trim = {"yes": True, "no": False}.get(args.trim, need_b > 0.9 * free)
    if trim:
        eng.trim()
        smp.mark("trim")
    recv = torch.empty(S * mx * rs, dtype=torch.uint8, device="cuda")
    slot = recv[R * mx * rs:(R + 1) * mx * rs]
    eng.export_edges(slot)
    dist.all_gather_into_tensor(slot, slot)   # world 1, in place
    for r in range(S):
        if r != R:
            recv[r * mx * rs:(r + 1) * mx * rs].copy_(slot)
    torch.cuda.synchronize()
    smp.mark("receive buffer filled")
    eng.import_edge_parts(recv, counts, mx)
    t["exchange_graph_s"] = round(time.perf_counter() - t0, 3)
    smp.mark("import + graph phase")
    del recv, slot
    torch.cuda.empty_cache()
    smp.mark("receive buffer freed")
    smp.stop.set()
    smp.t.join()
    tm2 = eng.timings()
    st = eng.stats()
    out = {"config": args.config, "rank": R, "shards": S, "resident_samples": len(need),
           "resident_gbp": round(sum(bases[s] for s in need) / 1e9, 2), "trim": trim,
           "edges_local": n, "edges_imported": n * S, "times": t,
           "device_peak_gb_sampled": round(smp.peak / 1e9, 2), "device_total_gb": round(smp.total / 1e9, 1),
           "engine_peak_gb": round(tm2["dev_peak_bytes"] / 1e9, 2),
           "engine_after_align_gb": round(tm["dev_bytes"] / 1e9, 2),
           "engine_now_gb": round(tm2["dev_bytes"] / 1e9, 2),
           "torch_max_allocated_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2),
           "torch_max_reserved_gb": round(torch.cuda.max_memory_reserved() / 1e9, 2),
           "hbm_model_gb": round(model[R] / 1e9, 2), "marks": smp.marks,
           "graph": {k: st[k] for k in ("edges", "components", "ideal_components")}}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "marks"}), flush=True)
    eng.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
