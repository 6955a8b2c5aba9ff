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
