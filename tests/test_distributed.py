"""The N > 1 path on CPU: two gloo ranks exchange their shards' edge records
(variable sizes, including an empty shard) exactly as the RCCL path does."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REC = 20   # sizeof(DEdge)


class SlotExchange:
    """Engine.export_edges(out) into this rank's slot of the padded receive
    buffer (a CPU tensor under gloo) and Engine.import_edge_parts over that
    buffer as it is (blocks of counts[r] records at stride `stride`): the
    exchange's exact sequence, in-place all-gather and padding included."""

    def export_edges(self, out=None):
        rec = self._records()
        if out is None:
            return rec.copy()
        assert out.numel() >= rec.size
        out.numpy()[:rec.size] = rec
        return rec.size // self.edge_record_size()

    def import_edge_parts(self, buf, counts, stride):
        rs = self.edge_record_size()
        b = buf.numpy() if hasattr(buf, "numpy") else np.asarray(buf)
        assert b.size >= len(counts) * stride * rs
        self.parts = list(counts)
        self.import_edges(np.concatenate([b[r * stride * rs:(r * stride + c) * rs] for r, c in enumerate(counts)]
                                         + [np.zeros(0, np.uint8)]))


class FakeShardEngine(SlotExchange):
    """The part of Engine the exchange touches; records are 20-byte blobs."""

    def __init__(self, rank, n):
        rng = np.random.default_rng(100 + rank)
        self.local = rng.integers(0, 256, n * REC, dtype=np.uint8)
        self.imported = None
        self.calls = []

    @staticmethod
    def edge_record_size():
        return REC

    def local_edge_count(self):
        return len(self.local) // REC

    def _records(self):
        return self.local

    def import_edges(self, buf, n=None):
        self.imported = np.asarray(buf).copy()

    def align(self):
        self.calls.append("align")

    def finish(self):
        self.calls.append("finish")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rna_clique_amd import distributed
        assert distributed.world() == (world, rank)
        eng = FakeShardEngine(rank, sizes[rank])
        distributed.sharded_run(eng)
        q.put((rank, eng.calls, eng.imported.tobytes(), eng.parts))
    finally:
        dist.destroy_process_group()


class FakeDustEngine(FakeShardEngine):
    """The part of Engine the DUST-mask exchange touches: a sample's mask is
    ceil(bases / 64) words, word i of sample s = s << 32 | i."""

    dust = (20, 64, 1)

    def __init__(self, rank, bases):
        super().__init__(rank, 1)
        self.bases = list(bases)
        self.made = None
        self.given = None

    def words(self, s):
        n = (self.bases[s] + 63) // 64
        return (np.uint64(s) << np.uint64(32)) | np.arange(n, dtype=np.uint64)

    def dust_masks(self, samples, out=None):
        assert out is None
        self.made = list(samples)
        return np.concatenate([self.words(s) for s in samples] + [np.zeros(0, np.uint64)])

    def set_dust_masks(self, samples, bits):
        self.given = (list(samples), np.asarray(bits).copy())


def _dust_worker(rank, world, port, bases, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rna_clique_amd import distributed
        eng = FakeDustEngine(rank, bases)
        distributed.exchange_dust(eng)
        q.put((rank, eng.made, eng.given[0], eng.given[1].tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bases", [(130, 64, 1, 0, 500, 7), (64, 64)])
def test_gloo_dust_exchange_world2(bases):
    """Every sample's DUST mask is made by exactly one rank that holds it, and
    after the all-gather every rank holds every mask, bit for bit."""
    from rna_clique_amd import distributed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dust_worker, args=(r, 2, port, bases, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, made, samples, blob = q.get(timeout=120)
        got[r] = (made, samples, blob)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    owner = distributed.dust_owners(list(bases), 2)
    order, first = distributed.plan_pairs(list(bases), 2)
    for r in range(2):
        held = {s for p in order[int(first[r]):int(first[r + 1])] for s in p}
        assert got[r][0] == [s for s in range(len(bases)) if owner[s] == r]
        assert set(got[r][0]) <= held
    made_all = got[0][0] + got[1][0]
    assert sorted(made_all) == sorted(s for s in range(len(bases)) if owner[s] >= 0)
    eng = FakeDustEngine(0, bases)
    want = np.concatenate([eng.words(s) for s in made_all] + [np.zeros(0, np.uint64)]).tobytes()
    for r in range(2):
        assert got[r][1] == made_all and got[r][2] == want


@pytest.mark.parametrize("sizes", [(3, 5), (7, 2), (0, 4), (0, 0)])
def test_gloo_edge_exchange_world2(sizes):
    """Unequal counts: each rank's records go into its slot of one padded
    buffer, gathered in place, imported as blocks at the largest count's
    stride."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, calls, blob, parts = q.get(timeout=120)
        got[r] = (calls, blob)
        assert parts == list(sizes)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = b"".join(FakeShardEngine(r, sizes[r]).local.tobytes() for r in range(2))
    for r in range(2):
        assert got[r][0] == ["align", "finish"]
        assert got[r][1] == want   # every rank sees all shards' edges, rank order


def test_world_without_init_is_single():
    from rna_clique_amd import distributed
    assert distributed.world() == (1, 0)


def test_plan_covers_every_pair_once_and_needed_samples():
    """rc_plan_pairs (no device): every pair in exactly one shard, and each
    shard's needed samples are exactly its pairs' samples (two ranges)."""
    from rna_clique_amd import distributed
    rng = np.random.default_rng(3)
    for n, shards in [(5, 2), (32, 8), (64, 8), (128, 8)]:
        bases = rng.integers(40_000_000, 60_000_000, size=n)
        order, first = distributed.plan_pairs(bases, shards)
        assert sorted(map(tuple, order)) == [(a, b) for a in range(n) for b in range(a + 1, n)]
        assert first[0] == 0 and first[-1] == len(order) and all(np.diff(first) >= 0)
        for r in range(shards):
            need = distributed.needed_samples(bases, shards, r)
            own = order[first[r]:first[r + 1]]
            assert need == {s for p in own for s in p}


def test_c5_fits_hbm_per_rank():
    """BASELINE C5 (128 samples x 100 000 genes, 200 bp - 5 kb transcripts,
    ~33 Gbp) on 8 GPUs: every rank's modelled HBM footprint (resident samples,
    one tile's working set, its HSP store, the group table) is within the
    288 GB of an MI355X, and within it with room to spare at the configuration's
    mean transcript length. (The model is calibrated on the engines' own
    device-memory peaks, r06: C3 59.9 GB, C4 177.2 GB, and the C5 rank of
    tests/test_gpu_scale.py 120.0 GB, which that test checks within 20 %.)"""
    from rna_clique_amd import distributed
    n, genes, mean_len = 128, 100_000, 2600
    bases = [genes * mean_len] * n
    fp = distributed.hbm_footprint(bases, [genes] * n, 8)
    assert max(fp) < 288e9, [f / 1e9 for f in fp]
    assert max(fp) < 0.72 * 288e9
    # sharding divides the resident bases and the HSP store
    one = distributed.hbm_footprint(bases, [genes] * n, 1)[0]
    assert max(fp) < 0.65 * one


class OracleShardEngine(SlotExchange):
    """The engine's sharded surface computed on the CPU oracles, so that the
    N > 1 host path runs on real alignments: its pairs from plan_pairs, DUST
    masks made by their owners and exchanged (each rank checks what it
    receives against its own), both directed searches and the gene matches
    table of each owned pair, the edges all-gathered, then the graph phase
    (components, ideal nodes) on every rank's edges and this rank's pair sums.
    Edge records are this stand-in's own 20-byte layout (the exchange moves
    opaque records)."""

    def __init__(self, samples, rank, world, dust=(20, 64, 1)):
        from oracle.align import OracleDB
        from rna_clique_amd import distributed
        self.samples = samples
        self.names = [s.name for s in samples]
        self.db = OracleDB(samples)
        self.bases = [int(s.seq.size) for s in samples]
        self.dust = dust
        order, first = distributed.plan_pairs(self.bases, world)
        self.pairs = [tuple(int(x) for x in p) for p in order[int(first[rank]):int(first[rank + 1])]]
        self.made, self.received_ok = [], None
        self.edges, self.sums = [], {}

    @staticmethod
    def edge_record_size():
        return 20

    def _mask_words(self, s):
        m = self.db.dust_mask(s, *self.dust).astype(np.uint8)
        m = np.concatenate([m, np.zeros(-m.size % 64, np.uint8)])
        return np.packbits(m, bitorder="little").view(np.uint64)

    def dust_masks(self, samples, out=None):
        assert out is None
        self.made = list(samples)
        return np.concatenate([self._mask_words(s) for s in samples] + [np.zeros(0, np.uint64)])

    def set_dust_masks(self, samples, bits):
        want = np.concatenate([self._mask_words(s) for s in samples] + [np.zeros(0, np.uint64)])
        self.received_ok = np.array_equal(np.asarray(bits, dtype=np.uint64), want)

    def align(self):
        from oracle import post_oracle
        from oracle.parity import hits_for_post
        for a, b in self.pairs:
            ora = {(q, s): self.db.align(q, s, 28, 108, 1e-99, False, self.dust) for q, s in ((a, b), (b, a))}
            hits = hits_for_post(self.samples, self.db, ora, self.names)
            t1, t2 = self.names[a], self.names[b]
            rows = post_oracle.match_table(post_oracle.parse_hits(hits[(t2, t1)], post_oracle.default_parse_id),
                                           post_oracle.parse_hits(hits[(t1, t2)], post_oracle.default_parse_id))
            self.sums[(a, b)] = rows
            for r in rows:
                self.edges.append((a, r["sgene"], b, r["qgene"]))

    def finish(self):
        pass

    def local_edge_count(self):
        return len(self.edges)

    def _records(self):
        rec = np.array([e + (0,) for e in self.edges], dtype=np.int32).reshape(-1, 5)
        return rec.view(np.uint8).reshape(-1)

    def import_edges(self, buf, n=None):
        from oracle import post_oracle
        rec = np.asarray(buf, dtype=np.uint8).view(np.int32).reshape(-1, 5)
        nodes, edges = set(), set()
        for sa, ga, sb, gb, _ in rec.tolist():
            u, v = (self.names[sa], ga), (self.names[sb], gb)
            nodes |= {u, v}
            edges.add(tuple(sorted((u, v))))
        valid = post_oracle.ideal_nodes(nodes, edges)
        self.sums = {(a, b): post_oracle.pair_sums(self.names[a], self.names[b], rows, valid)
                     for (a, b), rows in self.sums.items()}


def _oracle_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rna_clique_amd import distributed
        from rna_clique_amd.simulate import simulate
        samples, _ = simulate(4, 40, seed=77, p_iso2=0.2, indel_rate=0.003, polya=(0.3, 10, 40))
        eng = OracleShardEngine(samples, rank, world)
        distributed.sharded_run(eng)
        # every rank's pair sums to every rank (32-byte records)
        local = np.array([[a, b, n_, d_] for (a, b), (n_, d_) in sorted(eng.sums.items())],
                         dtype=np.int64).reshape(-1, 4)
        allt, total = distributed.all_gather_records(torch.from_numpy(local.view(np.uint8).reshape(-1)), 32)
        sums = allt.numpy()[:total * 32].view(np.int64).reshape(-1, 4).tolist()
        q.put((rank, eng.pairs, eng.made, eng.received_ok, sums))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_oracle_shards_match_one_process():
    """Two gloo ranks, each computing its planned pairs on the CPU oracle:
    after the DUST-mask exchange, the edge all-gather and the graph phase on
    every rank's edges, the ranks' pair sums give the one-process oracle's
    distance matrix exactly (the real-data counterpart of the FakeShardEngine
    tests; the GPU engine's own 2-rank path is test_gpu_api.py's RCCL test)."""
    from oracle import post_oracle
    from oracle.align import OracleDB
    from oracle.parity import hits_for_post, oracle_all_hsps
    from rna_clique_amd import distributed
    from rna_clique_amd.simulate import simulate
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_oracle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, pairs, made, ok, sums = q.get(timeout=300)
        got[r] = (pairs, made, ok, sums)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    samples, _ = simulate(4, 40, seed=77, p_iso2=0.2, indel_rate=0.003, polya=(0.3, 10, 40))
    names = [s.name for s in samples]
    bases = [int(s.seq.size) for s in samples]
    # the plan: every pair on exactly one rank; every mask made once, received intact
    assert sorted(got[0][0] + got[1][0]) == [(a, b) for a in range(4) for b in range(a + 1, 4)]
    owner = distributed.dust_owners(bases, 2)
    assert sorted(got[0][1] + got[1][1]) == sorted(s for s in range(4) if owner[s] >= 0)
    assert got[0][2] and got[1][2]
    assert got[0][3] == got[1][3] and len(got[0][3]) == 6
    # against the one-process oracle path
    db = OracleDB(samples)
    hits = hits_for_post(samples, db, oracle_all_hsps(db, 4, dust=(20, 64, 1), threads=4), names)
    res = post_oracle.run_pipeline(names, hits, post_oracle.default_parse_id)
    sums = {(names[a], names[b]): (n_, d_) for a, b, n_, d_ in got[0][3]}
    assert sums == res["sums"]
    lab_s, mat_s = post_oracle.distance_matrix(names, sums)
    lab_o, mat_o = post_oracle.distance_matrix(names, res["sums"])
    assert lab_s == lab_o and mat_s == mat_o
    assert len(res["valid"]) > 0
