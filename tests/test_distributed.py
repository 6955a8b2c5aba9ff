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


class FakeShardEngine:
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

    def export_edges(self, out=None):
        assert out is None
        return self.local.copy()

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
        q.put((rank, eng.calls, eng.imported.tobytes()))
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


@pytest.mark.parametrize("sizes", [(3, 5), (0, 4), (0, 0)])
def test_gloo_edge_exchange_world2(sizes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, calls, blob = q.get(timeout=120)
        got[r] = (calls, blob)
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
    mean transcript length. (The model is calibrated on the engine's own
    device-memory peak of rank 2 at C5, tests/test_gpu_scale.py: 202 GB
    measured device-wide in r03.)"""
    from rna_clique_amd import distributed
    n, genes, mean_len = 128, 100_000, 2600
    bases = [genes * mean_len] * n
    fp = distributed.hbm_footprint(bases, [genes] * n, 8)
    assert max(fp) < 288e9, [f / 1e9 for f in fp]
    assert max(fp) < 0.72 * 288e9
    # sharding divides the resident bases and the HSP store
    one = distributed.hbm_footprint(bases, [genes] * n, 1)[0]
    assert max(fp) < 0.65 * one
