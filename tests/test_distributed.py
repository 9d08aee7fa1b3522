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
    def rank(self, q, d, tgt_count, ks, row_offset):
        from oracle import retrieval as R
        s = R.scores(q.float().numpy(), d.float().numpy())
        h = R.hits(s, tgt_count, ks, row_offset).sum(0).astype(np.int64)
        return torch.from_numpy(h), torch.from_numpy(R.topk(s, max(ks))[0])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tables(fixture):
    from oracle.retrieval import bf16_to_f32
    if fixture == "retrieval":
        g = np.load(os.path.join(ROOT, "tests", "golden", "retrieval.npz"))
        return torch.from_numpy(bf16_to_f32(g["img"])), torch.from_numpy(bf16_to_f32(g["all_txt"]))
    from planted import planted_ties  # dense_ties.npz, case "narrow": exact duplicates across shards
    g = np.load(os.path.join(ROOT, "tests", "golden", "dense_ties.npz"))
    n, caps, D, seed = (int(x) for x in g["narrow_params"])
    img, allt, _ = planted_ties(n, caps, D, float(g["narrow_noise"]), seed)
    return img.float(), allt.float()


def _worker(rank, world, port, q, fixture="retrieval"):
    import sys
    for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd"), os.path.join(ROOT, "tests", "golden")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mme.distributed import shard_range, sharded_recall
    img, allt = _tables(fixture)
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


def test_sharded_recall_exact_ties_equals_reference(golden):
    """Exact ties across shard boundaries (duplicated images / captions, dense_ties.npz "narrow"): two
    ranks, each ranking its rows in torch.topk's order, reproduce compute_metrics_detailed's metrics."""
    g = golden("dense_ties")
    ref = dict(zip([str(k) for k in g["metric_names"]], g["narrow_metric_values"]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, "dense_ties")) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == ref


def test_shard_range_covers():
    from mme.distributed import shard_range
    for n in (1, 7, 5000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


# ------------------------------------------------------------------ ColPali (MaxSim) sharding
class MaxSimCPU:
    """CPU stand-in of the device MaxSim / top-k / hits with processor.score's bf16 semantics."""

    def maxsim(self, Q, ql, D, dl, flags):
        dots = torch.einsum("qid,njd->qnij", Q.float(), D.float()).to(torch.bfloat16).float()
        jmask = torch.arange(D.shape[1])[None, :] < dl[:, None].long()          # [n, Ld]
        dots = dots.masked_fill(~jmask[None, :, None, :], float("-inf"))
        m = dots.amax(-1)
        m = torch.where(flags.bool()[None, :, None], m.clamp_min(0.0), m)
        imask = torch.arange(Q.shape[1])[None, :] < ql[:, None].long()          # [q, Lq]
        m = m.masked_fill(~imask[:, None, :], 0.0)
        return m.sum(-1).to(torch.bfloat16).float()

    def recall(self, s, tgt_count, ks, row_offset):
        from oracle import torch_topk as TT
        return torch.from_numpy(TT.hits(s.numpy(), tgt_count, ks, row_offset).sum(0).astype(np.int64))


def _colpali_tables(n=13, caps=5, Ld=20, seed=0):
    """Planted per-item multi-vectors: image i tokens ~ base_i, its captions' tokens ~ base_i;
    captions left-padded per reference batch of 4 (pad = the batch-longest length)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(n, 128, generator=g)
    nrm = lambda x: (x / x.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    D = nrm(base[:, None] + 6.0 * torch.randn(n, Ld, 128, generator=g))
    lens = torch.randint(3, 10, (n * caps,), generator=g)
    Qa = torch.zeros(n * caps, 16, 128, dtype=torch.bfloat16)
    for c in range(n * caps):
        Qa[c, : lens[c]] = nrm(base[c // caps] + 6.0 * torch.randn(int(lens[c]), 128, generator=g))
    pad = torch.tensor([int(lens[s:s + 4].max()) for s in range(0, n * caps, 4) for _ in range(min(4, n * caps - s))])
    t2i = Qa[::caps].clone()
    t2i_len = lens[::caps].clone()
    return D, torch.full((n,), Ld, dtype=torch.int32), t2i, t2i_len.int(), Qa, lens.int(), pad.int()


def _colpali_worker(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mme.distributed import shard_range, sharded_colpali_recall
    D, dl, Qt, qtl, Qa, qal, qap = _colpali_tables()
    n, caps = D.shape[0], 5
    lo, hi = shard_range(n, rank, world)
    res = sharded_colpali_recall(D[lo:hi], dl[lo:hi], Qt[lo:hi], qtl[lo:hi], Qa[caps * lo:caps * hi],
                                 qal[caps * lo:caps * hi], qap[caps * lo:caps * hi], rank, world, n, caps,
                                 compute=MaxSimCPU())
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


def _reference_colpali_metrics():
    """The reference's colpali scoring (oracle/maxsim.py chunk loop over per-item lists whose
    caption tensors carry their left zero padding) + compute_metrics_detailed's recall."""
    from oracle import maxsim as om
    D, dl, Qt, qtl, Qa, qal, qap = _colpali_tables()
    n, caps = D.shape[0], 5

    def cap_items(Q, ql, qp):
        out = []
        for i in range(Q.shape[0]):
            e = torch.zeros(int(qp[i]), 128, dtype=torch.bfloat16)
            e[int(qp[i]) - int(ql[i]):] = Q[i, : int(ql[i])]
            out.append(e)
        return out
    t2i_pad = torch.tensor([int(qtl[s:s + 4].max()) for s in range(0, n, 4) for _ in range(min(4, n - s))])
    imgs = [D[i, : int(dl[i])] for i in range(n)]
    s_t2i = om.score_reference_chunks(cap_items(Qt, qtl, t2i_pad), imgs).numpy()
    s_i2t = om.score_reference_chunks(imgs, cap_items(Qa, qal, qap)).numpy()
    out = {}
    for name, s, tc in (("T2I", s_t2i, 1), ("I2T", s_i2t, caps), ("I2T_Sym", s_t2i.T.copy(), 1)):
        st = torch.from_numpy(s)
        for k in (1, 5, 10):  # compute_metrics_detailed: one torch.topk per row and k (main.py:331-378)
            hit = sum(any(c // tc == i for c in torch.topk(st[i], min(k, st.shape[1])).indices.tolist())
                      for i in range(n))
            out[f"{name}_R@{k}"] = 100.0 * hit / n
    return out


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_colpali_recall_equals_reference(world):
    ref = _reference_colpali_metrics()
    assert 0 < ref["T2I_R@1"] < 100  # planted data: recall neither trivial nor saturated
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_colpali_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == pytest.approx(ref)
