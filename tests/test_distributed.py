"""Multi-process sharding of the retrieval job on the CPU (gloo, world_size 2 and 3).

mme.distributed.sharded_recall is the orchestration bench.py runs over RCCL:
per-rank image shards (+ their captions), all-gather of the embedding tables,
ranking of each rank's own rows, all-reduce of the hit counters. Here the
compute callbacks are the numpy oracle; the result must equal the reference's
metrics on the golden planted fixture (tests/golden/retrieval.npz)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleOps:
    def topk(self, q, d, k):
        from oracle import retrieval as R
        idx, _ = R.topk(R.scores(q.float().numpy(), d.float().numpy()), k)
        return torch.from_numpy(idx)

    def hits(self, idx, tgt_count, ks, row_offset):
        from oracle import retrieval as R
        return torch.from_numpy(R.recall(idx.numpy(), tgt_count, ks, row_offset))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mme.distributed import shard_range, sharded_recall
    from oracle.retrieval import bf16_to_f32
    g = np.load(os.path.join(ROOT, "tests", "golden", "retrieval.npz"))
    img = torch.from_numpy(bf16_to_f32(g["img"]))
    allt = torch.from_numpy(bf16_to_f32(g["all_txt"]))
    n = img.shape[0]
    lo, hi = shard_range(n, rank, world)
    res = sharded_recall(img[lo:hi], allt[5 * lo:5 * hi:5], allt[5 * lo:5 * hi], rank, world, n, 5,
                         compute=OracleOps())
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_recall_equals_reference(golden, world):
    g = golden("retrieval")
    ref = dict(zip([str(k) for k in g["metric_names"]], g["metric_values"]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == pytest.approx(ref)


def test_shard_range_covers():
    from mme.distributed import shard_range
    for n in (1, 7, 5000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
