"""Multi-GPU: one engine per GPU, sample pairs sharded, one edge exchange.

SURVEY.md §8e. rc_plan_pairs gives every rank one rectangle [a0, a1) x
[b0, b1) of the (a, b) pair triangle, chosen by recursive bisection against a
cost model of pair work and per-sample work (query-word lookups, index), so
each rank's samples are two short contiguous ranges. A rank holds the
sequences of those samples only (`needed_samples`; the others are added as
metadata: transcripts and genes, no bases), aligns its pairs -- both directed
searches, in tiles of at most 2^32 bases when its samples do not fit one
pass -- and runs top-N / reciprocal best hits for them, which yields its share
of the gene matches tables and graph edges. The ideal-clique filter needs the
whole graph, so the edge records (20 B each: two node ids, the pair, and the
edge's nident and length - gaps sums) are all-gathered once -- over RCCL on
GPUs, gloo on CPU -- and every rank runs connected components, the ideal
filter and the pair sums over all of them. Before the alignment the ranks
exchange DUST masks (each sample masked once, by one rank that holds it:
dust_owners / exchange_dust), so the query-side masking does not repeat on
every rank that holds a sample. These two all-gathers are the only
collectives on the data path.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat


def world(process_group=None):
    """(world size, rank) of an initialised torch.distributed group, else (1, 0)."""
    try:
        import torch.distributed as dist
    except ImportError:
        return 1, 0
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(process_group), dist.get_rank(process_group)


def plan_shards(sample_bases, shard_count):
    """pair_first[shard_count + 1] from rc_plan_shards (no device needed)."""
    return plan_pairs(sample_bases, shard_count)[1]


def plan_pairs(sample_bases, shard_count):
    """([(a, b), ...] the pair order, pair_first[shard_count + 1]) from
    rc_plan_pairs (no device needed)."""
    b = np.ascontiguousarray(sample_bases, dtype=np.int64)
    n = len(b)
    m = n * (n - 1) // 2
    pa, pb = np.zeros(max(m, 1), dtype=np.int32), np.zeros(max(m, 1), dtype=np.int32)
    out = np.zeros(shard_count + 1, dtype=np.int64)
    nat.check(nat.lib().rc_plan_pairs(b.ctypes.data_as(ctypes.c_void_p), n, int(shard_count),
                                      pa.ctypes.data_as(ctypes.c_void_p), pb.ctypes.data_as(ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p)))
    return list(zip(pa[:m].tolist(), pb[:m].tolist())), out


def needed_samples(sample_bases, shard_count, rank):
    """The samples whose sequences rank `rank` needs: those of its pairs."""
    order, first = plan_pairs(sample_bases, shard_count)
    out = set()
    for a, b in order[int(first[rank]):int(first[rank + 1])]:
        out.add(a)
        out.add(b)
    return out


def _tiles(pairs, sample_bases, tile_bases):
    """The alignment tiles of a rank's pairs, as the engine plans them
    (engine.hip plan_tiles): one tile when its samples fit `tile_bases`, else
    every (a chunk, b chunk) with pairs, chunks of at most half the cap."""
    U = sorted({s for p in pairs for s in p})
    if sum(sample_bases[s] for s in U) <= tile_bases:
        return [pairs]

    def chunks(R):
        out, acc = [[]], 0
        for s in R:
            if out[-1] and acc + sample_bases[s] > tile_bases // 2:
                out.append([])
                acc = 0
            out[-1].append(s)
            acc += sample_bases[s]
        return out
    CA = chunks(sorted({a for a, _ in pairs}))
    CB = chunks(sorted({b for _, b in pairs}))
    ia = {s: i for i, c in enumerate(CA) for s in c}
    ib = {s: j for j, c in enumerate(CB) for s in c}
    tiles = {}
    for a, b in pairs:
        tiles.setdefault((ia[a], ib[b]), []).append((a, b))
    return list(tiles.values())


# device bytes per candidate slot of a tile: the record (48), both directed
# searches' first-seed results (2 x 48), HSP slots (2 x 56), counts and
# overflow offsets, defer / wide lists, ~10 seeds of 12 B; capacities grow by
# 1.25x (calibrated on the engines' measured peaks, r06: C3 59.9 GB, C4
# 177.2 GB, a C5 rank 120.0 GB)
CAND_BYTES = 525


def hbm_footprint(sample_bases, sample_genes, shard_count, tile_bases=(1 << 32) - (1 << 24),
                  hsps_per_gene=1.0):
    """Modelled device bytes of every rank (a planning aid: bench and tests
    check that a configuration fits 288 GB per GPU before running it; the
    engine reports what it actually holds, rc_timing.dev_peak_bytes). Per rank:
    * its samples' bases, resident (1 B/base; the array grows by 1.25x);
    * the largest alignment tile's working set (`_tiles`: the engine's tile
      plan): the tile's gathered copy (1 B/base), packed forward + reverse
      complement (0.5), transcript-start and DUST bit arrays (0.25), the
      near-mask index (0.5); the 16-mer index and its sort buffer over the
      tile's subject samples only (16 B/base); its candidates (one per gene of
      each pair, CAND_BYTES each); the 2^28-bucket table (1 GiB);
    * its HSP store (56 B per HSP, both directed searches of every pair; the
      store grows by 1.5x) and table rows (16 B each);
    * the (gene, sample) group table over all genes x samples (8 B: offset,
      count); each tile's group counts and scans are part of its working set;
    * per (pair, gene) RBH item 100 B (row and edge slots, counts, offsets)
      and the edge records (20 B) of all ranks after the exchange."""
    import math
    order, first = plan_pairs(sample_bases, shard_count)
    n = len(sample_bases)
    genes = sum(sample_genes)
    out = []
    for r in range(shard_count):
        pairs = order[int(first[r]):int(first[r + 1])]
        samples = {s for p in pairs for s in p}
        resident = sum(sample_bases[s] for s in samples)
        work = 0
        for tp in _tiles(pairs, sample_bases, tile_bases):
            tile = sum(sample_bases[s] for s in {s for p in tp for s in p})
            subj = sum(sample_bases[s] for s in {b for _, b in tp})
            cands = sum(min(sample_genes[a], sample_genes[b]) for a, b in tp)
            # the tile's group counts and scans (12 B each): direct groups of
            # its query genes x every sample, mirrored ones of its subject
            # genes x its query samples
            A, B = {a for a, _ in tp}, {b for _, b in tp}
            gcount = 12 * (sum(sample_genes[a] for a in A) * n + sum(sample_genes[b] for b in B) * len(A))
            work = max(work, tile * (1 + 0.5 + 0.25 + 0.5) + subj * 16 + cands * CAND_BYTES + gcount + (1 << 30))
        nh = sum(sample_genes[a] + sample_genes[b] for a, b in pairs) * hsps_per_gene
        items = sum(sample_genes[b] for a, b in pairs)
        groups = genes * n * 8
        edges = sum(min(sample_genes[a], sample_genes[b]) for a, b in order) * 20
        out.append(int(1.25 * resident + work + nh * (56 * 1.5 + 16) + items * 100 + groups + edges
                       + math.comb(n, 2) * 64))
    return out


def all_gather_records(local, record_size, process_group=None, device=None):
    """Variable-length all-gather of fixed-size records.

    `local` is a uint8 tensor (CUDA for RCCL, CPU for gloo) holding this
    rank's records. Returns (concatenation of every rank's records in rank
    order, record count). Sizes go first, then one padded all-gather."""
    import torch
    import torch.distributed as dist
    W = dist.get_world_size(process_group)
    dev = local.device if device is None else device
    n = torch.tensor([local.numel() // record_size], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(W)]
    dist.all_gather(counts, n, group=process_group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts) * record_size
    if mx == 0:
        return torch.zeros(0, dtype=torch.uint8, device=dev), 0
    if local.numel() == mx:
        send = local
    else:
        send = torch.zeros(mx, dtype=torch.uint8, device=dev)
        send[:local.numel()] = local
    if dist.get_backend(process_group) == "gloo":
        recv = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(W)]
        dist.all_gather(recv, send, group=process_group)
    else:
        # RCCL: one receive buffer (no per-rank tensors), views into it
        buf = torch.empty(W * mx, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(buf, send, group=process_group)
        recv = list(buf.view(W, mx))
        if all(c * record_size == mx for c in counts):
            return buf, sum(counts)   # no padding anywhere: the buffer is the result
    out = torch.cat([r[:c * record_size] for r, c in zip(recv, counts)])
    return out, sum(counts)


def exchange_edges(eng, process_group=None, trim=None):
    """All-gather the shards' graph edges and run the graph phase on them.
    The engine must have run align() and finish().

    The counts go first; each rank's records are exported straight into its
    own slot of one padded receive buffer (W x the largest count), gathered in
    place, and the engine imports that buffer as it is (rc_import_edge_parts:
    no compacting copy). RCCL: a device buffer, device-to-device throughout;
    gloo: the same buffer in host memory (the CPU tests run this exact
    sequence: slot aliasing, padding, unequal counts). `trim`: free the
    engine's alignment working set first (rc_trim) -- None = only when the
    receive buffer, the imported records and the graph writer's sort buffers
    would not fit in free device memory (C5: 17 GB + 16 GB beside a ~146 GB
    alignment working set)."""
    import torch
    import torch.distributed as dist
    rs = eng.edge_record_size()
    on_gpu = dist.get_backend(process_group) != "gloo" and torch.cuda.is_available()
    dev = "cuda" if on_gpu else "cpu"
    W, R = world(process_group)
    n = eng.local_edge_count()
    c = torch.tensor([n], dtype=torch.int64, device=dev)
    cs = [torch.zeros_like(c) for _ in range(W)]
    dist.all_gather(cs, c, group=process_group)
    counts = [int(x.item()) for x in cs]
    mx = max(counts)
    if on_gpu and trim is None:
        free, _ = torch.cuda.mem_get_info()
        trim = exchange_device_bytes(counts, rs) > 0.9 * free
    if on_gpu and trim:
        eng.trim()
    recv = torch.empty(max(W * mx * rs, 1), dtype=torch.uint8, device=dev)
    if mx:
        mine = recv[R * mx * rs:(R + 1) * mx * rs]
        eng.export_edges(mine)             # into this rank's slot (device-to-device on GPUs)
        dist.all_gather_into_tensor(recv[:W * mx * rs], mine, group=process_group)
        if on_gpu:
            torch.cuda.current_stream().synchronize()   # the engine runs on its own stream
    eng.import_edge_parts(recv, counts, mx)
    del recv
    if on_gpu and mx * W * rs >= (1 << 30):
        torch.cuda.empty_cache()   # the engine allocates outside torch's pool


def exchange_device_bytes(counts, record_size):
    """Device bytes the edge exchange and the graph phase after it add on top
    of an engine's alignment working set: the imported copy of every record,
    plus the larger of the padded receive buffer (W x the largest count; freed
    after the import) and what rc_write_graph then allocates for the device
    sort of the records (16 B of keys and indices per record, a sorted record
    copy, and the radix sort's scratch, about its key bytes)."""
    W, mx, tot = len(counts), max(counts) if counts else 0, sum(counts)
    return tot * record_size + max(W * mx * record_size, tot * (16 + record_size + 8))


def dust_owners(sample_bases, shard_count):
    """The rank that makes each sample's DUST mask (-1: no rank holds it):
    one of the ranks holding the sample, the one with the fewest bases
    assigned so far, largest samples first -- so every mask is computed once
    and the work is spread over the ranks."""
    order, first = plan_pairs(sample_bases, shard_count)
    n = len(sample_bases)
    holders = [set() for _ in range(n)]
    for r in range(shard_count):
        for a, b in order[int(first[r]):int(first[r + 1])]:
            holders[a].add(r)
            holders[b].add(r)
    load = [0] * shard_count
    owner = [-1] * n
    for s in sorted(range(n), key=lambda s: (-int(sample_bases[s]), s)):
        if holders[s]:
            r = min(holders[s], key=lambda r: (load[r], r))
            owner[s] = r
            load[r] += int(sample_bases[s])
    return owner


def exchange_dust(eng, process_group=None, force=False):
    """Every sample's DUST mask made once: this rank masks the samples
    dust_owners gives it, the masks are all-gathered (1 bit per base; 200 MB
    at C3) and each engine takes them (rc_set_dust_masks) instead of masking
    its resident samples itself. A no-op without DUST or with one rank
    (`force`: run the exchange on a one-rank group too -- the tests' way to
    drive the device path on a one-GPU box)."""
    import torch
    import torch.distributed as dist
    W, R = world(process_group)
    if (W == 1 and not force) or getattr(eng, "dust", None) is None:
        return
    owner = dust_owners(eng.bases, W)
    mine = [s for s in range(len(owner)) if owner[s] == R]
    everyone = [s for r in range(W) for s in range(len(owner)) if owner[s] == r]
    on_gpu = dist.get_backend(process_group) != "gloo" and torch.cuda.is_available()
    if on_gpu:
        nw = sum((eng.bases[s] + 63) // 64 for s in mine)
        local = torch.empty(max(nw, 1), dtype=torch.int64, device="cuda")[:nw]
        eng.dust_masks(mine, local)
        allt, total = all_gather_records(local.view(torch.uint8), 8, process_group)
        torch.cuda.current_stream().synchronize()
        eng.set_dust_masks(everyone, allt.contiguous().view(torch.int64)[:total])
    else:
        local = torch.from_numpy(eng.dust_masks(mine).view(np.uint8))
        allt, total = all_gather_records(local, 8, process_group)
        eng.set_dust_masks(everyone, allt.numpy().view(np.uint64))


def sharded_run(eng, process_group=None, trim=None):
    """rc_run for a sharded engine: DUST masks made once across the ranks,
    align + RBH locally, exchange (`trim`: see exchange_edges), graph."""
    exchange_dust(eng, process_group)
    eng.align()
    eng.finish()
    exchange_edges(eng, process_group, trim=trim)
