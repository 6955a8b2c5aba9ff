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
