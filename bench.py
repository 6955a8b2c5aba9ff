"""Benchmark: sample-pairs/s of the whole pairwise-distance path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]

One step = one pass of the hot path over the whole synthetic batch with the
inputs already resident in HBM: 2-bit pack -> seed index build -> seed-and-
extend for every directed sample pair -> top-N + reciprocal best hits -> gene
matches graph + ideal-clique filter -> restricted sums -> N x N distance matrix
copied to the host. For N > 1 GPUs (torch.distributed.run, one rank per GPU)
the sample pairs are sharded by sequence length (rc_plan_shards), every rank
aligns its pairs and runs reciprocal best hits for them, the graph edges are
exchanged with one RCCL all-gather, and every rank finishes the graph.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline
model and the CPU baseline.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the wall-clock leg (FASTA files -> rna_clique() -> matrix.h5)")
    ap.add_argument("--cpu-pairs", type=int, default=1,
                    help="sample pairs the CPU baseline times (2 directed searches each)")
    return ap.parse_args()


def algorithmic_bytes(samples, hsps_per_pair, word=28):
    """B_pair = 8 (P_A + P_B) + (L_A + L_B) / 4 + 32 H_pair,
    summed over all C(N, 2) pairs (P_X = seed positions at word size `word`)."""
    import numpy as np
    P, L = [], []
    for s in samples:
        lens = np.diff(s.tx_offsets.astype(np.int64))
        P.append(int(np.maximum(lens - word + 1, 0).sum()))
        L.append(int(lens.sum()))
    n = len(samples)
    tot = 0
    for a in range(n):
        for b in range(a + 1, n):
            tot += 8 * (P[a] + P[b]) + (L[a] + L[b]) / 4
    return tot + 32 * hsps_per_pair


def traffic_from_profile(config, world):
    """HBM bytes per step of the seed + extend kernels from the committed PMC
    profile (profiles/<round>/<config>_pmc.json, FETCH_SIZE doubled per the
    gfx950 note + WRITE_SIZE; collected with scripts/gpu_pmc.sh), or None."""
    import glob
    if world != 1:
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"{config}_pmc.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("traffic_bytes_seed_extend")


def cpu_baseline(samples, n_pairs=1):
    """The C oracle (same algorithm, one core) on a bounded sample of the same
    workload: `n_pairs` sample pairs, both directed searches each, plus the
    post-alignment oracle on them. Returns pairs/s."""
    from oracle.align import OracleDB
    from oracle import post_oracle
    from oracle.parity import hits_for_post
    t0 = time.perf_counter()
    done = 0
    for k in range(n_pairs):
        a, b = 2 * k, 2 * k + 1
        sub = [samples[a], samples[b]]
        db = OracleDB(sub)
        hs = {(0, 1): db.align(0, 1), (1, 0): db.align(1, 0)}
        hits = hits_for_post(sub, db, hs)
        names = [s.name for s in sub]
        post_oracle.run_pipeline(names, hits, post_oracle.default_parse_id)
        done += 1
    dt = time.perf_counter() - t0
    return done / dt, dt


def e2e_wall_clock(samples, genes, rank, world, dist, ref):
    """The metric's second half: wall-clock from the transcripts FASTA files on
    disk to matrix.h5 written, through the drop-in API -- rna_clique() with
    top-gene selection (native FASTA reader, od1/*_top.fasta written), engine
    load + H2D, the whole GPU path, the distance matrix and the h5 writer.
    The FASTA files are written (untimed) to a scratch directory first; the
    gene matches tables and graph.pkl are not written (out_dir_2 /
    output_graph None). `ref` = (labels, matrix) of the timed steps: the
    matrix must come out identical."""
    import shutil
    import numpy as np
    from rna_clique_amd.rna_clique import rna_clique, last_timings
    base = os.environ.get("RC_E2E_DIR", "/tmp")
    root = os.path.join(base, f"rc_e2e_{os.getppid() if world > 1 else os.getpid()}")
    dirs = [os.path.join(root, "in", s.name) for s in samples]
    t_w = time.perf_counter()
    if rank == 0:
        for s, d in zip(samples, dirs):
            os.makedirs(d, exist_ok=True)
            s.write_fasta(os.path.join(d, "transcripts.fasta"))
    t_w = time.perf_counter() - t_w
    if dist:
        dist.barrier()
    od1 = os.path.join(root, f"od1_r{rank}")
    out = os.path.join(root, "matrix.h5")
    t0 = time.perf_counter()
    sim, pts = rna_clique(dirs, od1, None, None, None, out, top_genes=genes,
                          jobs=16)
    dt = time.perf_counter() - t0
    if dist:
        import torch
        dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    df = sim.get_dissimilarity_df()
    name_of = {str(p): n for p, n in pts.items()}
    order = [name_of[str(l)] for l in df.index]
    labels, mat = ref
    idx = [list(labels).index(n) for n in order]
    same = bool(np.array_equal(df.to_numpy(), np.asarray(mat)[np.ix_(idx, idx)]))
    size = os.path.getsize(out) if rank == 0 else None
    if dist:
        dist.barrier()
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    return {"wall_clock_s": round(dt, 3), "matrix_h5_bytes": size, "matrix_equal_to_steps": same,
            "fasta_write_s": round(t_w, 1),
            "phases_s": {k: round(v, 3) for k, v in last_timings.items()},
            "what": "transcripts FASTA on disk -> top-gene selection -> GPU path -> matrix.h5 "
                    "(gene matches tables and graph.pkl not written)"}


def main():
    args = parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch as _t
    ndev = max(1, _t.cuda.device_count())
    device = local_rank % ndev   # one GPU per rank; ranks share a GPU only in rehearsals
    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    from rna_clique_amd import distributed
    from rna_clique_amd.engine import Engine
    from rna_clique_amd.simulate import simulate, CONFIGS
    cfg = CONFIGS[args.config]
    t_gen = time.perf_counter()
    samples, _ = simulate(**cfg)
    t_gen = time.perf_counter() - t_gen
    n = len(samples)
    pairs = n * (n - 1) // 2
    eng = Engine(device=device, shard_rank=rank, shard_count=world)
    for s in samples:
        eng.add_sample(s.name, s.seq, s.tx_offsets, s.gene, s.iso)
    eng.upload()   # inputs resident in HBM before timing (H2D excluded)

    def step():
        if world == 1:
            eng.run()
        else:
            distributed.sharded_run(eng)
        return eng.distance()

    for _ in range(args.warmup):
        step()
    kern_ms = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        labels, mat = step()
        tmi = eng.timings()
        kern_ms.append(tmi["seed_kernel_ms"] + tmi["align_kernel_ms"])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if args.backend != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = 1e3 * dt / args.steps
    value = pairs * args.steps / dt
    st = eng.stats()
    tm = eng.timings()
    e2e = None
    if not args.no_e2e:
        eng.close()   # free this engine's HBM before rna_clique() builds its own
        e2e = e2e_wall_clock(samples, cfg["genes"], rank, world, dist, (labels, mat))
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    # roofline of the dominant kernel pair (seed + extend), SURVEY.md §8d byte
    # model over this rank's share of the pairs; time = HIP events on the
    # engine's stream around the two launches
    hsps = st["hsps"]
    avg_k = sum(kern_ms) / len(kern_ms)
    bytes_launch = algorithmic_bytes(samples, hsps) * (1.0 / world)
    achieved = bytes_launch / (avg_k * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic_from_profile(args.config, world),
            "kernel": "seed_kernel + extend_kernel", "kernel_ms": round(avg_k, 3),
            "bytes_per_launch": int(bytes_launch)}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        v, secs = cpu_baseline(samples, args.cpu_pairs)
        cpu = {"value": round(v, 5), "unit": "sample-pairs/s", "cores": 1, "kind": "port",
               "sample": f"{args.cpu_pairs} of {pairs} {args.config} sample pairs "
                         f"(2 directed searches each + RBH/graph oracle), {secs:.1f} s"}
    line = {
        "metric": "sample-pairs/sec (all-vs-all alignment -> RBH graph -> distance matrix)",
        "value": round(value, 3), "unit": "sample-pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u8/int32", "data": "synthetic (simulate.py, seeded, BASELINE configs)",
        "config": {"workload": f"{args.config}: {n} samples x {cfg['genes']} genes",
                   "pairs": pairs, "bases": int(sum(s.seq.size for s in samples)),
                   "parallelism": f"sample-pair shards x{world}"},
        "roofline": roof, "cpu_baseline": cpu, "wall_clock_to_matrix": e2e,
        "phases_ms": {k: round(v, 3) for k, v in tm.items()},
        "graph": {k: st[k] for k in ("seeds", "candidates", "hsps", "table_rows", "edges", "components",
                                     "ideal_components", "sample_count")},
        "gen_s": round(t_gen, 1),
    }
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
