"""The RCCL branch of the sharded job's exchange on a real GPU.

bench.py's N > 1 runs all-gather the embedding tables with all_gather_into_tensor and all-reduce
the hit counters over the "nccl" backend (RCCL on ROCm). A one-GPU box cannot hold two RCCL ranks
(RCCL refuses two ranks on one device; the same-device rehearsals use gloo), so this runs the same
collectives — mme.distributed._gather_ragged (row-count exchange, padded gather, strip) and
all_reduce_ — in a one-rank RCCL group on cuda:0, in a child process so the group's resources end
with it."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from test_distributed import ROOT, _free_port

pytestmark = pytest.mark.gpu


def _rccl_worker(port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from mme.distributed import _gather_ragged, all_reduce_
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(7, 1152, generator=g, device="cuda").to(torch.bfloat16)
        y = _gather_ragged(x, 1)
        counts = torch.arange(9, dtype=torch.int64, device="cuda")
        all_reduce_(counts, dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        q.put((dist.get_backend(), bool(torch.equal(x, y)), y.shape == x.shape, counts.tolist()))
    finally:
        dist.destroy_process_group()


def test_rccl_gather_and_reduce_one_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    p.join(120)
    if p.is_alive():
        p.kill()
        pytest.fail("RCCL worker did not finish within 120 s")
    assert p.exitcode == 0, f"RCCL worker exit code {p.exitcode}"
    backend, same, shape_ok, counts = q.get(timeout=5)
    print(f"backend {backend}: gathered rows identical {same}, counters {counts}")
    assert backend == "nccl" and same and shape_ok and counts == list(range(9))
