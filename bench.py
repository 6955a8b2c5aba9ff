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
    ap.add_argument("--cpu-pairs", type=int, default=0,
                    help="sample pairs the CPU baseline times (2 directed searches each; "
                         "default 2 x the worker count)")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="CPU baseline processes (default: the usable cores, at most 16)")
    ap.add_argument("--shard", default=None, metavar="R/S",
                    help="emulate rank R of an S-GPU run on this one GPU: only that rank's samples are "
                         "generated and resident, its pairs aligned (align + RBH timed); prints a "
                         "shard_emulation line (C5 on a 1-GPU box)")
    return ap.parse_args()


def launch_ranks(args):
    """`--gpus N` without an outer launcher: run N ranks of this script under
    torch.distributed.run as a CHILD process (nothing here has touched the
    GPU; no exec) and pass rank 0's JSON line through. Returns the exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    proc = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    # rank 0's JSON line on stdout; anything else the ranks printed there
    # (gloo / RCCL banners) goes to stderr
    for line in proc.stdout.splitlines():
        print(line, file=sys.stdout if line.startswith("{") else sys.stderr, flush=True)
    return proc.returncode


def src_hash():
    """Hash of the engine's sources (csrc + the C ABI header): profiles under
    profiles/ carry it, and a PMC figure is only reported for the sources it
    was measured on."""
    import hashlib
    h = hashlib.sha256()
    base = os.path.join(ROOT, "rna_clique_amd", "csrc")
    for name in sorted(os.listdir(base)):
        with open(os.path.join(base, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    with open(os.path.join(ROOT, "include", "rcgpu.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


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


def pmc_profile(config, world):
    """The newest committed PMC summary (profiles/<tag>/<config>_pmc.json,
    scripts/pmc_summary.py) measured on these very sources, or None."""
    import glob
    if world != 1:
        return None
    h = src_hash()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"{config}_pmc.json")), reverse=True):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("src_hash") == h:
            d["file"] = os.path.relpath(f, ROOT)
            return d
    return None


def issue_roofline(iss, align_kernel_ms):
    """The extension's issue roofline: it is bound by VALU issue, not bytes.
    The row kernel's VALU instructions per step (PMC summary `issue`) over
    that kernel's own time per step (kernel trace of the same sources, when
    the summary has it; else every extension kernel's live HIP-event time, an
    upper bound) against the VALU issue peak (a wave64 instruction holds a
    32-lane SIMD for 2 clocks)."""
    own = iss.get("kernel_ms")
    t_ext = (own if own else align_kernel_ms) * 1e-3
    peak = iss.get("valu_peak_g_per_s", 256 * 4 * 2.4 / 2)
    return {"bound": "valu", "unit": "G wave-VALU/s",
            "achieved": round(iss["valu"] / t_ext / 1e9, 1), "peak": peak,
            "frac": round(iss["valu"] / t_ext / 1e9 / peak, 4),
            "salu_g_per_s": round(iss["salu"] / t_ext / 1e9, 1),
            "valu_per_wave_step": iss.get("valu_per_wave_step"),
            "kernel": iss.get("kernel", "extend_rows_kernel"),
            "kernel_ms": round(t_ext * 1e3, 3),
            "kernel_ms_source": iss.get("kernel_ms_source") if own else "live extension kernels (HIP events)"}


def binding(prof, issue):
    """What the PMC profile of these very sources says binds the two hot
    kernels: the seed kernel's share of wave cycles spent waiting, the row
    kernel's VALU issue fraction. Only written when such a profile exists."""
    out = {}
    sk = prof.get("kernels", {}).get("seed_kernel", {})
    if sk.get("SQ_WAVE_CYCLES"):
        w = sk["SQ_WAIT_ANY"] / sk["SQ_WAVE_CYCLES"]
        out["seed_kernel"] = f"waves wait {100 * w:.0f}% of their cycles (SQ_WAIT_ANY / SQ_WAVE_CYCLES, {prof['file']})"
    if issue:
        out["extend_rows_kernel"] = f"VALU issue at {100 * issue['frac']:.0f}% of peak (issue_extension)"
    return out


_CPU_SAMPLES = None


def _cpu_pair(ab):
    """One sample pair on the CPU port: both directed searches (C oracle) and
    the post-alignment path (RBH, table) -- a worker of cpu_baseline."""
    from oracle.align import OracleDB
    from oracle import post_oracle
    from oracle.parity import hits_for_post
    a, b = ab
    sub = [_CPU_SAMPLES[a], _CPU_SAMPLES[b]]
    db = OracleDB(sub)
    hs = {(0, 1): db.align(0, 1, dust=(20, 64, 1)), (1, 0): db.align(1, 0, dust=(20, 64, 1))}
    names = [s.name for s in sub]
    post_oracle.run_pipeline(names, hits_for_post(sub, db, hs), post_oracle.default_parse_id)
    return ab


def cpu_baseline(samples, workers, n_pairs):
    """The CPU port of the same algorithm (oracle/: the C alignment oracle and
    the post-alignment oracle) on `workers` processes, one sample pair per
    task, over `n_pairs` of the workload's pairs. Runs before the GPU is
    initialised (forked workers). Returns (pairs/s, seconds)."""
    import itertools
    import multiprocessing as mp
    global _CPU_SAMPLES
    _CPU_SAMPLES = samples
    pairs = list(itertools.combinations(range(len(samples)), 2))
    step = max(1, len(pairs) // n_pairs)
    todo = pairs[::step][:n_pairs]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(workers) as pool:
        done = len(list(pool.imap_unordered(_cpu_pair, todo)))
    dt = time.perf_counter() - t0
    return done / dt, dt, done


def cpu_workers(samples, forced=0):
    """(processes, how chosen) for the CPU baseline: every core this process
    may use (affinity mask and cgroup quota, oracle.parity.usable_cores),
    unless host memory cannot hold that many concurrent pair tasks (a task
    holds a subject index of 24 B per seed position while it sorts it, and
    the two samples' base codes)."""
    import numpy as np
    from oracle.parity import usable_cores
    uc = usable_cores()
    if forced:
        return forced, dict(uc, forced=forced)
    P = max(int(np.maximum(np.diff(s.tx_offsets.astype(np.int64)) - 15, 0).sum()) for s in samples)
    L = max(int(s.tx_offsets[-1]) for s in samples)
    per_task = 24 * P + 2 * L + (64 << 20)
    try:
        import psutil
        avail = psutil.virtual_memory().available
    except ImportError:
        avail = 64 << 30
    # the GPU box caps one command at ~270 GiB of host memory
    budget = int(0.6 * min(avail, 250 << 30))
    by_mem = max(1, budget // per_task)
    n = max(1, min(uc["cores"], by_mem))
    return n, dict(uc, memory_cap=int(by_mem), task_bytes=int(per_task))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def e2e_wall_clock(samples, genes, rank, world, dist, ref):
    """The metric's second half: wall-clock from the transcripts FASTA files on
    disk to matrix.h5 written, through the drop-in API -- rna_clique() with
    top-gene selection (native FASTA reader, od1/*_top.fasta written), engine
    load + H2D, the whole GPU path, and every output the reference writes:
    the od2 gene matches tables (pandas table-format HDF5), graph.pkl and
    matrix.h5. The FASTA files are written (untimed) to a scratch directory
    first. `ref` = (labels, matrix) of the timed steps: the matrix must come
    out identical."""
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
    od2, graph = os.path.join(root, f"od2_r{rank}"), os.path.join(root, f"graph_r{rank}.pkl")
    sim, pts = rna_clique(dirs, od1, od2, None, graph, out, top_genes=genes, jobs=16)
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
    n_tables = len(os.listdir(od2))
    graph_mb = round(os.path.getsize(graph) / 1e6, 1) if rank == 0 else None
    if dist:
        dist.barrier()
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
    return {"wall_clock_s": round(dt, 3), "to_matrix_h5_s": round(last_timings.get("to_matrix_s", dt), 3),
            "matrix_h5_bytes": size, "matrix_equal_to_steps": same,
            "od2_tables": n_tables, "graph_pkl_mb": graph_mb, "fasta_write_s": round(t_w, 1),
            "phases_s": {k: round(v, 3) for k, v in last_timings.items()},
            "what": "transcripts FASTA on disk -> top-gene selection -> GPU path -> od2/*.h5 gene matches "
                    "tables + graph.pkl + matrix.h5 (every output the reference writes)"}


def shard_samples(config, shard_count, rank):
    """(samples, needed sample set, pair plan) of rank `rank` of a
    `shard_count`-GPU run of `config`: with the config's per-node random
    streams only the rank's own samples are generated (C5: ~17 of 33 Gbp),
    the others come back as metadata (seq None)."""
    from rna_clique_amd import distributed
    from rna_clique_amd.simulate import simulate, CONFIGS
    cfg = dict(CONFIGS[config])
    if cfg.get("node_rng"):
        meta, _ = simulate(only=[], **cfg)
        bases = [int(s.tx_offsets[-1]) for s in meta]
        need = distributed.needed_samples(bases, shard_count, rank)
        del meta
        samples, _ = simulate(only=sorted(need), **cfg)
    else:
        samples, _ = simulate(**cfg)
        bases = [int(s.tx_offsets[-1]) for s in samples]
        need = distributed.needed_samples(bases, shard_count, rank)
    return samples, need, distributed.plan_pairs(bases, shard_count)


def shard_emulation(args):
    """--shard R/S: rank R's share of an S-GPU run on this one GPU (the pool
    gives one GPU per box; the driver runs the real S-GPU bench). Only the
    rank's samples are generated and resident; its pairs are aligned and go
    through top-N / reciprocal best hits (align + finish: the rank's whole
    data-parallel work), timed; then the graph phase runs on the rank's own
    edges. Prints one shard_emulation JSON line: the rank's pairs/s, tiles,
    measured HBM use vs distributed.hbm_footprint's model."""
    R, S = (int(x) for x in args.shard.split("/"))
    # torch's HIP runtime first, then librcgpu.so (the shard plan below loads
    # it): the other order leaves the engine's runtime without a device
    import torch
    torch.cuda.init()
    from rna_clique_amd import distributed
    t_gen = time.perf_counter()
    samples, need, (order, first) = shard_samples(args.config, S, R)
    t_gen = time.perf_counter() - t_gen
    bases = [int(s.tx_offsets[-1]) for s in samples]
    genes = [len(set(s.gene.tolist())) for s in samples]
    model = distributed.hbm_footprint(bases, genes, S)
    my_pairs = int(first[R + 1] - first[R])
    free0, total = torch.cuda.mem_get_info(0)
    from rna_clique_amd.engine import Engine
    eng = Engine(device=0, shard_rank=R, shard_count=S)
    for i, s in enumerate(samples):
        eng.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
    del samples
    eng.upload()
    cold = []   # the warmup calls: the first one allocates every device buffer
    for _ in range(args.warmup):
        t0 = time.perf_counter()
        eng.align()
        eng.finish()
        cold.append(round(time.perf_counter() - t0, 3))
        tmc = eng.timings()
        cold_phases = {k: round(tmc[k], 1) for k in ("load_ms", "align_wall_ms", "host_wait_ms", "index_ms",
                                                      "seed_kernel_ms", "align_kernel_ms", "dust_ms")}
        print(json.dumps({"warmup_s": cold[-1], "phases_ms": cold_phases}), flush=True)
    times = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        eng.align()
        eng.finish()
        times.append(time.perf_counter() - t0)
    tm = eng.timings()
    free1, _ = torch.cuda.mem_get_info(0)
    t0 = time.perf_counter()
    eng.import_edges(eng.export_edges())   # the graph phase on this rank's own edges
    t_graph = time.perf_counter() - t0
    st = eng.stats()
    dt = sum(times) / len(times)
    line = {"metric": "shard_emulation: one rank's sample pairs/s (align + top-N/RBH of its pairs)",
            "config": args.config, "rank": R, "shard_count": S, "pairs": my_pairs,
            "total_pairs": len(order), "resident_samples": len(need),
            "resident_bases": int(sum(bases[i] for i in need)),
            "value": round(my_pairs / dt, 3), "unit": "sample-pairs/s", "s_per_step": round(dt, 3),
            "cold_s": cold, "warm_s": [round(x, 3) for x in times],
            "steps": args.steps, "warmup": args.warmup,
            "projected_job_pairs_per_s_if_balanced": round(len(order) / dt, 1),
            "hbm_used_gb": round((free0 - free1) / 1e9, 2), "hbm_total_gb": round(total / 1e9, 1),
            "engine_peak_gb": round(tm["dev_peak_bytes"] / 1e9, 2),
            "hbm_model_gb": round(model[R] / 1e9, 2), "hbm_model_max_rank_gb": round(max(model) / 1e9, 2),
            "graph_own_edges_s": round(t_graph, 3), "gen_s": round(t_gen, 1),
            "phases_ms": {k: round(v, 3) for k, v in tm.items()},
            "graph": {k: st[k] for k in ("seeds", "candidates", "hsps", "table_rows", "edges", "components",
                                         "ideal_components")}}
    print(json.dumps(line), flush=True)
    eng.close()
    return 0


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.shard:
        sys.exit(shard_emulation(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    import numpy as np
    from rna_clique_amd import distributed
    from rna_clique_amd.simulate import simulate, CONFIGS
    cfg = CONFIGS[args.config]
    t_gen = time.perf_counter()
    samples, _ = simulate(**cfg)
    t_gen = time.perf_counter() - t_gen
    n = len(samples)
    pairs = n * (n - 1) // 2
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the CPU port on this host's cores, before anything touches the GPU
        # (the device count below included: the pool's workers are forked)
        workers, why = cpu_workers(samples, args.cpu_workers)
        n_cpu = args.cpu_pairs or max(8, workers)
        v, secs, done = cpu_baseline(samples, workers, n_cpu)
        cpu = {"value": round(v, 4), "unit": "sample-pairs/s", "cores": workers, "kind": "port",
               "cpu": cpu_model(), "extrapolated": True, "cores_how": why,
               "sample": f"{done} of {pairs} {args.config} sample pairs (both directed searches with DUST "
                         f"+ reciprocal best hits / table each, one pair per process, {workers} processes) "
                         f"in {secs:.1f} s; pairs/s extrapolated to the whole workload"}
    import torch
    ndev = max(1, torch.cuda.device_count())
    device = local_rank % ndev   # one GPU per rank; ranks share a GPU only in rehearsals
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    from rna_clique_amd.engine import Engine
    eng = Engine(device=device, shard_rank=rank, shard_count=world)
    # a rank holds the sequences of its own pairs' samples only
    need = distributed.needed_samples([int(s.tx_offsets[-1]) for s in samples], world, rank) \
        if world > 1 else set(range(n))
    for i, s in enumerate(samples):
        eng.add_sample(s.name, s.seq if i in need else None, s.tx_offsets, s.gene, s.iso)
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
    # roofline of the dominant kernel pair (seed + extension), SURVEY.md §8d
    # byte model over this rank's share of the pairs; time = HIP events on
    # the engine's stream around those launches
    hsps = st["hsps"]
    avg_k = sum(kern_ms) / len(kern_ms)
    bytes_launch = algorithmic_bytes(samples, hsps) * (1.0 / world)
    achieved = bytes_launch / (avg_k * 1e-3) / 1e9
    prof = pmc_profile(args.config, world)
    traffic = prof.get("traffic_bytes_seed_extend") if prof else None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            # the counters' bytes over the same kernel time: the HBM bandwidth
            # actually moved (achieved/frac above use the byte model, per contract)
            "measured_gbs": round(traffic / (avg_k * 1e-3) / 1e9, 1) if traffic else None,
            "measured_frac": round(traffic / (avg_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
            "traffic_source": prof["file"] if prof else "no PMC profile of these sources (src_hash "
                                                       f"{src_hash()})",
            "kernel": "seed_kernel + extension kernels", "kernel_ms": round(avg_k, 3),
            "bytes_per_launch": int(bytes_launch),
            # what achieved/frac are, and what actually binds these kernels
            # (DESIGN.md §4): neither is at an HBM wall
            "achieved_is": "SURVEY.md 8d algorithmic bytes (a model) / live kernel time"}
    if prof and prof.get("issue"):
        roof["issue_extension"] = issue_roofline(prof["issue"], tm["align_kernel_ms"])
    if prof:
        roof["binding"] = binding(prof, roof.get("issue_extension"))
    if cpu:
        cpu["gpu_speedup"] = round(value / cpu["value"], 1)
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
