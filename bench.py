#!/usr/bin/env python3
"""Headline benchmark: SigLIP-400M, 5 000 images x 25 000 captions, end to end.

Metric (BASELINE.json): images/sec for the whole job — encode n images
(224x224x3 u8 -> PIL-exact bicubic 384 -> ViT), n T2I captions and 5n
captions (SigLIP text, L = 64), L2-normalise, the 5k x 5k and 5k x 25k
similarity + top-k, and Recall@{1,5,10} (T2I, I2T, I2T-Sym) — the v28
definition of the reference's published QPS
(run_benchmark_grand_slam_v28_publication_ready.py:305-408; A40: 47.1 img/s,
benchmark_v28_all_models_combined.csv:7). One "step" = one such job.
Inputs are synthetic (u8 images + token ids) and already resident in HBM
when the timed region starts; weights are seeded random init at the exact
architecture (no checkpoints offline).

Multi-GPU: launched by torch.distributed.run, one process per GPU; each rank
encodes its image shard + the captions of those images (no collective), then
all-gathers embeddings (RCCL) and ranks its rows against the full tables;
hit counters are all-reduced. value = images of the whole job / max-rank time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from mme.config import exec_batches  # noqa: E402  (no HIP call: the library loads lazily)

A40_PUBLISHED_IMG_S = 47.1  # SigLIP-400M end-to-end img/s, A40 bf16 bs32
A40_COLPALI_IMG_S = 2.9     # ColPali-v1.3 img/s (encoder + MaxSim), A40 bf16 bs4 (5k job)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
MFMA_FP8_PEAK_TFLOPS = 5000.0  # dense fp8 (block-scaled f8f6f4 MFMA)
HBM_PEAK_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (default: the launcher's WORLD_SIZE under torchrun, else 1)")
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="SigLIP-400M")
    p.add_argument("--n-images", type=int, default=None, help="images of the job (default 5 000; ColPali 1 000)")
    p.add_argument("--caps", type=int, default=5)
    p.add_argument("--img-batch", type=int, default=None,
                   help="images per vision-tower batch before the tail-aware split (default mme.config.exec_batches: "
                        "EXEC_IMG_BATCH; ColPali 32)")
    p.add_argument("--txt-batch", type=int, default=None,
                   help="captions per text-tower batch before the tail-aware split (default mme.config.exec_batches: "
                        "EXEC_TXT_BATCH, SigLIP EXEC_TXT_BATCH_SIGLIP; ColPali 2048)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-kernel-timer", action="store_true")
    p.add_argument("--no-parity", action="store_true",
                   help="skip the post-run R@1 parity check of the job's embeddings against the oracle")
    p.add_argument("--no-host-inputs", dest="host_inputs", action="store_false",
                   help="skip the extra job whose u8 images start in host memory (streamed H2D, SURVEY 8f-2; "
                        "the reference's timed region includes its host processor + H2D, main.py:407,534-559); "
                        "reported as host_inputs_img_s, never as value")
    p.add_argument("--bootstrap", type=int, default=0,
                   help="also time N bootstrap resamples of the recall on the device (main.py:586-634; untimed "
                        "by the headline metric, reported separately)")
    p.add_argument("--backend", default="nccl", help="process-group backend for N > 1 (nccl = RCCL on ROCm; "
                   "gloo = rehearsal of the multi-rank path, e.g. with --same-device)")
    p.add_argument("--same-device", action="store_true",
                   help="every rank on cuda:0 (rehearse N ranks on a one-GPU box; needs --backend gloo)")
    p.add_argument("--fp8", action="store_true",
                   help="mx8 encoder GEMMs (BASELINE configs[4]: DFN5B-H fp8 weights on the fp8 MFMA)")
    p.add_argument("--gemm-form", type=int, default=None,
                   help="A/B only: run every GEMM call with this libmme kernel form (mme.ops.kernel_forms; "
                        "47 = pipe6, 93 = the run-time-branched epilogues, 95 = pipe10 on every non-split shape); "
                        "reported on the line")
    p.add_argument("--mx-form", type=int, default=None,
                   help="A/B only: run every mx8 GEMM call with this libmme mx kernel form (mme.ops.kernel_forms; "
                        "11 = mx11, 15 = mx11 with the bias loaded up front); reported on the line")
    p.add_argument("--attn-form", type=int, default=None,
                   help="A/B only: run every attention call with T > 128 (the vision towers; text attention keeps "
                        "the production dispatch) with this libmme kernel form (mme.ops.kernel_forms "
                        "attention_long; 30 + kind forces a kernel kind); reported on the line")
    return p.parse_args()


def synth_inputs(spec, n, caps, device):
    """Deterministic synthetic job on the device: u8 images [n,224,224,3], ids [caps*n, L]."""
    g = torch.Generator(device=device)
    g.manual_seed(0)
    imgs = torch.randint(0, 256, (n, 224, 224, 3), generator=g, device=device, dtype=torch.uint8)
    t = spec.text
    L = t.max_pos
    g.manual_seed(1)
    if t.bos_id is not None:
        body = torch.randint(1, min(t.bos_id, t.eos_id), (caps * n, L - 2), generator=g, device=device)
        ids = torch.cat([torch.full((caps * n, 1), t.bos_id, device=device), body,
                         torch.full((caps * n, 1), t.eos_id, device=device)], 1)
    else:
        body = torch.randint(2, t.vocab, (caps * n, L - 1), generator=g, device=device)
        ids = torch.cat([body, torch.full((caps * n, 1), t.eos_id, device=device)], 1)
    return imgs, ids.to(torch.int64)


HBM_FAMILIES = {  # KernelTimer family -> the kernel(s) behind it (rocprof names)
    "preprocess": "resample_patch_p_kernel", "rowstats": "rowstats_kernel", "layernorm": "layernorm_kernel",
    "l2norm": "l2norm_kernel", "attention_short": "attn_short_kernel", "attention_short2": "attn_short2_kernel"}


def load_traffic(model, n, img_batch, txt_batch, fp8):
    """profiles/hbm_traffic.json (tools/pmc_job.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over one job,
    tools/pmc_summary.py) when it was measured on this configuration, else None."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    want = {"model": model, "n_images": n, "img_batch": img_batch, "txt_batch": txt_batch, "fp8": bool(fp8)}
    for entry in d.get("configs", []):
        if all(entry.get("config", {}).get(k) == v for k, v in want.items()):
            return dict(entry["families"], _source=f"profiles/hbm_traffic.json ({entry.get('build', '?')})")
    return None


def hbm_rooflines(kt, dt, pmc, steps):
    """HBM-bound kernels of the job: algorithmic bytes per launch / HIP-event time of the
    timed launches vs the 8 TB/s peak, and the PMC-measured bytes per launch where the pass matches."""
    out = {}
    for fam, kname in HBM_FAMILIES.items():
        if fam not in kt:
            continue
        k = kt[fam]
        gbs = k["bytes"] / (k["ms"] / 1e3) / 1e9
        r = {"kernel": kname, "launches_per_job": k["launches"] // max(steps, 1),
             "avg_launch_ms": round(k["ms"] / k["launches"], 4),
             "algorithmic_bytes_per_launch": round(k["bytes"] / k["launches"]),
             "achieved_GBs": round(gbs, 1), "peak_GBs": HBM_PEAK_GBS, "frac": round(gbs / HBM_PEAK_GBS, 4),
             "share_of_step_time": round(k["ms"] / 1e3 / dt, 4)}
        m = (pmc or {}).get(kname)
        if m and abs(m.get("launches", 0) - r["launches_per_job"]) <= 0.005 * r["launches_per_job"]:
            r["traffic"] = round(m["hbm_bytes_per_launch"])
            r["traffic_GBs"] = round(m["hbm_bytes_per_launch"] / (r["avg_launch_ms"] / 1e3) / 1e9, 1)
        out[fam] = r
    return out


def cpu_baseline(spec, seconds: float, tables=None, caps_per_image: int = 5):
    """The oracle's bf16 PyTorch-CPU restatement of the reference encoders (validated against the
    reference's own main.encode_data in profiles/r02_cpu_baseline_check.json) at the reference's
    batch size 32 (main.py:73,395), timed on the host cores on a bounded sample: whole batches of
    images and captions until the time budget is spent (at least one of each), extrapolated to the
    job's n images + 6n captions; plus the CPU retrieval of the job itself (oracle/retrieval.py:
    fp32 matmul + top-10 in torch.topk's order + recall, main.py:471-473,331-378), timed in full on the job's
    own embedding tables."""
    from oracle import encoders as oe
    from oracle import retrieval as R
    from mme.processor import synthetic_caption_ids, synthetic_images
    from mme.weights import random_state_dict
    sd = {k: v.cpu() for k, v in random_state_dict(spec, seed=0, device="cuda").items()}
    threads = torch.get_num_threads()
    bs = 32
    imgs = synthetic_images(4 * bs)
    caps = synthetic_caption_ids(spec, 32 * bs).tolist()

    def run(fn, items, budget):
        done, t0 = 0, time.time()
        while done < len(items) and (done == 0 or (time.time() - t0) < budget):
            fn(items[done:done + bs])
            done += len(items[done:done + bs])
        return done, time.time() - t0

    oe.encode_data(spec, sd, list(imgs[:1]), caps[:1], bs=1)  # warm the allocator / threads
    ni, ti = run(lambda x: oe.encode_data(spec, sd, list(x), [], bs=bs), imgs, seconds * 0.6)
    nc, tc = run(lambda x: oe.encode_data(spec, sd, [], x, bs=bs), caps, seconds * 0.25)
    img_s, cap_s = ni / ti, nc / tc
    ret_s, n = 0.0, None
    if tables is not None:
        img, t2i, allc = (tables[k].float().cpu().numpy() for k in ("img", "t2i", "all"))
        n = img.shape[0]
        t0 = time.time()
        for q, d, tc_ in ((t2i, img, 1), (img, allc, caps_per_image), (img, t2i, 1)):
            R.hits(R.scores(q, d), tc_).sum(0)
        ret_s = time.time() - t0
    per_img = 1.0 / img_s + 6.0 / cap_s + (ret_s / n if n else 0.0)
    return {"value": round(1.0 / per_img, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/encoders.py bf16 CPU, bs {bs}: {ni} images in {ti:.1f}s ({img_s:.2f} img/s) + "
                      f"{nc} captions in {tc:.1f}s ({cap_s:.2f} cap/s), extrapolated to n images + 6n captions; "
                      f"+ oracle retrieval of the job's own {n} x {caps_per_image * n if n else 0} tables "
                      f"(T2I + I2T + Sym, top-10 + recall) {ret_s:.2f}s, timed in full",
            "encode_img_s": round(img_s, 4), "encode_cap_s": round(cap_s, 3), "retrieval_s": round(ret_s, 3)}


def retrieval_parity(tables, metrics, caps_per_image: int = 5):
    """R@1 parity of the headline job (checker; runs after the timed region): the job's own
    embedding tables ranked on the device (mme.retrieval.rank_rows: fused sim/top-11, exact-tie rows
    re-selected in torch.topk's CPU order) vs the oracle (numpy fp32 matmul + torch.topk's order,
    oracle/retrieval.py restating main.py:471-473 and 331-378), row by row; the job's device recall
    vs the oracle's recall of the same tables (one selection per k, as compute_metrics_detailed)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import retrieval as R
    from mme.retrieval import rank_rows
    t0 = time.time()
    host = {k: tables[k].float().cpu().numpy() for k in ("img", "t2i", "all")}
    n = host["img"].shape[0]
    rows = {}
    ref_metrics = {}
    for name, qk, dk, tc in (("T2I", "t2i", "img", 1), ("I2T", "img", "all", caps_per_image),
                             ("I2T_Sym", "img", "t2i", 1)):
        k = min(10, host[dk].shape[0])  # the reference clamps k to the column count (main.py:335)
        ranked = rank_rows(tables[qk], tables[dk], tc)
        s = R.scores(host[qk], host[dk])
        ridx, _ = R.topk(s, k)
        _, rsc = R.topk(s, k + 1)
        tied = np.zeros(len(ridx), bool)
        tied[ranked.tie_rows.cpu().numpy()] = True
        only, missed = [], []
        same, near = R.compare_topk(ranked.idx.cpu().numpy(), ridx, rsc, exact_rows=tied,
                                    dev_score=ranked.score.cpu().numpy(), oracle_only=only, unflagged=missed)
        rows[name] = {"rows_identical": f"{int(same.sum())}/{len(same)}", "near_tie_rows": int(near.sum()),
                      "decisive_rows_differing": int((~same & ~near).sum()),
                      "exact_tie_rows_torch_order": int(ranked.tie_rows.numel()),
                      "oracle_only_exact_tie_rows": len(only), "device_ties_unflagged": len(missed)}
        for kr, h in zip((1, 5, 10), R.hits(s, tc).sum(0)):
            ref_metrics[f"{name}_R@{kr}"] = 100.0 * h / n
    return {"recall_identical": all(ref_metrics[k] == metrics[k] for k in ref_metrics),
            "oracle_recall": {k: round(v, 2) for k, v in ref_metrics.items()}, "rows": rows,
            "near_tie_rule": "neighbouring oracle scores among the top 11 within 1e-5*|s1|; exact ties are not "
                             "exempt on rows the device finds tied too (torch.topk's order, replayed on both "
                             "sides); an oracle-only exact tie is a near tie (counted in oracle_only_exact_tie_rows); "
                             "a device row whose own top-11 scores tie must be flagged by tie_rows "
                             "(device_ties_unflagged, 0 expected)",
            "checker": "oracle/retrieval.py on the job's own embeddings (numpy fp32 + torch.topk order, host)",
            "seconds": round(time.time() - t0, 2)}


def fp8_drift(model_name, dev, imgs, t2i_ids, cap_ids, fp8_tables, img_batch, txt_batch, caps: int = 5):
    """fp8 against bf16 over the WHOLE job (checker; after the timed region, --fp8 only): the same
    weights (seed 0) loaded without the mx8 GEMMs encode the job's images and captions, and the
    job's fp8 tables are compared with them (mme.mx.job_drift: per-row cosine of the embeddings; the
    T2I, I2T (every image against all 5n captions) and I2T_Sym rankings, mme_sim_topk, as top-1 agreement on
    the rows decided beyond the measured fp8 score perturbation (gated, with the decided counts), and the I2T
    agreement over all rows plus top-10 overlap (reported); `drift_ok` against mme.mx.JOB_DRIFT_BOUNDS, which
    tests/test_gpu_mx.py asserts on the same job)."""
    from mme import mx
    from mme.models import load_model
    t0 = time.time()
    bf, _ = load_model(model_name, seed=0, device=dev, fp8=False)
    bf_tables = {"img": bf.encode_images(imgs, batch=img_batch), "t2i": bf.encode_texts(t2i_ids, exec_batch=txt_batch),
                 "all": bf.encode_texts(cap_ids, exec_batch=txt_batch)}
    del bf
    d = mx.job_drift(fp8_tables, bf_tables)
    torch.cuda.synchronize()
    d.update(checker="the same weights in bf16 (mme, no mx8 GEMMs) over the whole job", seconds=round(time.time() - t0, 2))
    return d


def encoder_parity(spec, imgs_u8, cap_ids, dev_img, dev_txt, bar: float = 0.999):
    """Encoder parity of the headline job (checker; after the timed region): the job's own images and
    T2I captions at the first, middle and last rows encoded by the fp32 oracle (oracle/encoders.py: the PIL-exact processor and the
    transformers towers restated, validated against main.encode_data) with the job's own weights,
    against the device embeddings the job produced (cosine per item; the SURVEY §8d bar is 0.999, 0.99 for
    the mx-fp8 encoder GEMMs)."""
    sys.path.insert(0, ROOT)
    from oracle import encoders as oe
    from mme.weights import random_state_dict
    t0 = time.time()
    sd = {k: v.float().cpu() for k, v in random_state_dict(spec, seed=0, device="cuda").items()}
    oi, ot = oe.encode_data(spec, sd, list(imgs_u8.cpu().numpy()), cap_ids.cpu().tolist(), bs=len(imgs_u8),
                            out_dtype=torch.float32)
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a.float().cpu(), b.float(), dim=-1)
    ci, ct = cos(dev_img, oi), cos(dev_txt, ot)
    return {"items": int(len(imgs_u8)), "img_cos_min": round(float(ci.min()), 6), "txt_cos_min": round(float(ct.min()), 6),
            "bar": bar, "ok": bool(ci.min() >= bar and ct.min() >= bar),
            "checker": "oracle/encoders.py fp32 on the job's own images / T2I captions (rows listed) and weights",
            "seconds": round(time.time() - t0, 2)}


def colpali_encoder_parity(imgs_u8, t2i_caps, tables, img_batch: int = 32, bar_min: float = 0.995,
                           bar_mean: float = 0.999):
    """ColPali encoder parity of the job (checker; after the timed region): the job's own images at the
    first and last rows of its first execution batch and the job's last image, and its first and last
    T2I queries (each in its reference batch of 4, left-padded as process_queries, main.py:420-425),
    encoded by the fp32 oracle (oracle/colpali_encoder.py) with the job's weights, against the
    device's multi-vectors: per-token cosine (mean >= 0.999; min >= 0.995)."""
    sys.path.insert(0, ROOT)
    from oracle import colpali_encoder as oc
    from mme.colpali_encoder import random_state_dict
    from mme.config import COLPALI
    t0 = time.time()
    spec = COLPALI["ColPali-v1.3"]
    sd = {k: v.float().cpu() for k, v in random_state_dict(spec, seed=0, device="cuda").items()}
    n = imgs_u8.shape[0]
    img_rows = sorted({0, min(img_batch, n) - 1, n - 1})
    D, dl, Qt, qtl = (tables[k] for k in ("D", "dl", "Qt", "qtl"))
    cos = lambda a, b: torch.nn.functional.cosine_similarity(a.float().cpu(), b.float(), dim=-1)
    res = {"image_rows": img_rows, "query_rows": sorted({0, len(t2i_caps) - 1})}
    ci = [cos(D[i, : int(dl[i])], oc.encode_image(spec, sd, imgs_u8[i].cpu().numpy())) for i in img_rows]
    cq = []
    for i in res["query_rows"]:
        lo = i // spec.batch_size * spec.batch_size
        ref = oc.encode_query_batch(spec, sd, t2i_caps[lo:lo + spec.batch_size])[i - lo]
        cq.append(cos(Qt[i, : int(qtl[i])], ref))
    c = torch.cat(ci + cq)
    res.update(img_cos_min=round(float(torch.cat(ci).min()), 6), query_cos_min=round(float(torch.cat(cq).min()), 6),
               cos_mean=round(float(c.mean()), 6), bar_min=bar_min, bar_mean=bar_mean,
               ok=bool(c.min() >= bar_min and c.mean() >= bar_mean),
               checker="oracle/colpali_encoder.py fp32 on the job's own images / T2I queries and weights",
               seconds=round(time.time() - t0, 2))
    return res


def colpali_parity(tables, scores, caps_per_image: int = 5, n_t2i: int = 50, n_i2t: int = 10, n_sym: int = 50,
                   imgs_u8=None, t2i_caps=None):
    """MaxSim parity of the ColPali job (checker; runs after the timed region): sampled query rows
    of the job's own multi-vector tables re-scored on the host by the oracle's restatement of the
    reference's colpali chunk loop (oracle/maxsim.py: pad_sequence + bf16 einsum / max / sum per
    10-doc chunk, main.py:451-470 -> processor.score), against the device's score rows: scores
    bit-identical, top-10 columns identical in torch.topk's CPU order (oracle/torch_topk.cpp vs the
    device's mme_topk_rows_torch; MaxSim sums are bf16-quantised, so exact ties are common) and the
    rows' hit / miss at k = 1, 5, 10 identical, one selection per k (main.py:331-378). Rows:
    T2I (caption-0 queries vs all images), I2T (image queries vs all caption docs, each with its
    batch's left padding), I2T-Sym (= T2I columns: every T2I query against one image)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import maxsim as om
    from oracle import torch_topk as TT
    from mme import ops
    t0 = time.time()
    D, dl, Qt, qtl, qtp, Qa, qal, qap = (tables[k] for k in ("D", "dl", "Qt", "qtl", "qtp", "Qa", "qal", "qap"))
    n = D.shape[0]
    dlh, qtlh, qtph, qalh, qaph = (x.cpu().tolist() for x in (dl, qtl, qtp, qal, qap))
    Dh, Qth, Qah = D.cpu(), Qt.cpu(), Qa.cpu()

    def items(Q, ql, qp):  # per-item [L_b, 128] with its leading zero rows, as encode_data returns them
        out = []
        for i in range(Q.shape[0]):
            e = torch.zeros(qp[i], Q.shape[2], dtype=Q.dtype)
            e[qp[i] - ql[i]:] = Q[i, : ql[i]]
            out.append(e)
        return out
    img_items = [Dh[i, : dlh[i]] for i in range(n)]
    t2i_items, cap_items = items(Qth, qtlh, qtph), items(Qah, qalh, qaph)
    rng = np.random.default_rng(7)
    out, ok = {}, True
    for name, m, tc in (("T2I", n_t2i, 1), ("I2T", n_i2t, caps_per_image), ("I2T_Sym", n_sym, 1)):
        rows = np.sort(rng.choice(n, min(m, n), replace=False))
        if name == "T2I":
            ref = om.score_reference_chunks([t2i_items[r] for r in rows], img_items)
            dev = scores["t2i"][torch.from_numpy(rows).to(scores["t2i"].device)]
        elif name == "I2T":
            ref = torch.cat([om.score_reference_chunks([img_items[r]], cap_items) for r in rows])
            dev = scores["i2t"][torch.from_numpy(rows).to(scores["i2t"].device)]
        else:
            ref = torch.cat([om.score_reference_chunks(t2i_items, [img_items[r]]) for r in rows], 1).t()
            dev = scores["t2i"][:, torch.from_numpy(rows).to(scores["t2i"].device)].t()
        ref = ref.numpy().astype(np.float32)
        dev = dev.contiguous()
        ks = [min(kk, ref.shape[1]) for kk in (1, 5, 10)]
        didx = {kk: ops.topk_rows_torch(dev, kk)[0].cpu().numpy() for kk in ks}
        ridx = {kk: TT.topk(ref, kk)[0] for kk in ks}
        hit = lambda ix: np.stack([(ix[kk] // tc == rows[:, None]).any(1) for kk in ks], 1)
        dev = dev.cpu().numpy()
        ulp = np.abs(torch.from_numpy(dev).to(torch.bfloat16).view(torch.int16).int().numpy()
                     - torch.from_numpy(ref).to(torch.bfloat16).view(torch.int16).int().numpy())
        top11 = lambda x: -np.sort(-x, 1)[:, :11]
        same_top = (top11(dev) == top11(ref)).all(1)
        same_idx = (didx[ks[-1]] == ridx[ks[-1]]).all(1)
        same_hit = (hit(didx) == hit(ridx)).all(1)
        r = {"rows_sampled": int(len(rows)), "scores_max_ulp": int(ulp.max()),
             "scores_identical_frac": round(float((ulp == 0).mean()), 6),
             "rows_top11_identical": int(same_top.sum()), "top10_identical": int(same_idx.sum()),
             "hit_rows_identical": int(same_hit.sum())}
        # a CPU bf16 GEMM and the MFMA sum a dot product's 128 fp32 products in different orders, so a
        # score may round 1 bf16 ulp apart; every row whose top-11 values agree must rank identically
        ok &= r["scores_max_ulp"] <= 1 and bool((same_idx | ~same_top).all()) and bool((same_hit | ~same_top).all())
        out[name] = r
    return {"parity_ok": bool(ok), "rows": out,
            "encoders": colpali_encoder_parity(imgs_u8, t2i_caps, tables) if imgs_u8 is not None else None,
            "rule": "scores <= 1 bf16 ulp apart; rows whose top-11 agree: top-10 in torch.topk's CPU order and "
                    "hit/miss at k = 1, 5, 10 identical",
            "checker": "oracle/maxsim.py chunk loop (reference main.py:451-470) on the job's own multi-vectors, host",
            "full_geometry_pin": "tests/test_gpu_colpali.py::test_colpali_full_geometry_vs_reference "
                                 "(1 000 x 5 000 vs the reference's own scores and recall)",
            "seconds": round(time.time() - t0, 2)}


def colpali_captions(n: int, caps: int, seed: int = 1):
    """Synthetic caption token lists for the ColPali job: 8..14 ids each, so a query is
    1 + 3 + len + 10 + 1 = 23..29 tokens (Tq ~ 26)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = rng.integers(8, 15, n * caps)
    return [rng.integers(3, 250000, int(L)).tolist() for L in lens]


def cpu_baseline_colpali(spec, seconds: float, n: int = 1000, caps: int = 5):
    """oracle/colpali_encoder.py (bf16 PyTorch-CPU) on a bounded sample: images and
    queries timed separately, extrapolated to n images + 6n queries; plus the reference's
    MaxSim chunk loop (oracle/maxsim.py, 10 x 10 chunks, main.py:451-470) timed on sample
    chunks of the job's shapes and extrapolated to its (n/10)^2 T2I + (n/10)(5n/10) I2T calls."""
    import numpy as np
    from oracle import colpali_encoder as oc
    from oracle import pil_bicubic
    from mme.colpali_encoder import random_state_dict
    from mme.processor import synthetic_images
    sd = {k: v.cpu() for k, v in random_state_dict(spec, seed=0, device="cuda").items()}
    threads = torch.get_num_threads()
    ip = spec.image_proc
    imgs = synthetic_images(4)
    qcaps = colpali_captions(64, 1)

    def enc_img(a):
        pv = torch.from_numpy(pil_bicubic.normalize(pil_bicubic.preprocess_u8(a, ip.size, ip.mode), ip.mean,
                                                    ip.std))[None]
        oc.forward(spec, sd, torch.tensor([spec.image_tokens]), None, pv)

    def enc_q(batch):
        rows = [list(spec.query_tokens(c)) for c in batch]
        L = max(len(r) for r in rows)
        ids = torch.full((len(rows), L), spec.pad_id, dtype=torch.int64)
        m = torch.zeros_like(ids)
        for i, r in enumerate(rows):
            ids[i, L - len(r):] = torch.tensor(r)
            m[i, L - len(r):] = 1
        oc.forward(spec, sd, ids, m)

    t0, ni = time.time(), 0
    while ni < len(imgs) and (ni == 0 or time.time() - t0 < seconds * 0.7):
        enc_img(imgs[ni])
        ni += 1
    ti = time.time() - t0
    t0, nc = time.time(), 0
    while nc < len(qcaps) and (nc == 0 or time.time() - t0 < seconds * 0.3):
        enc_q(qcaps[nc:nc + 4])
        nc += 4
    tc = time.time() - t0
    from oracle import maxsim as om
    g = torch.Generator().manual_seed(0)
    docs = [torch.randn(len(spec.image_tokens), 128, generator=g).to(torch.bfloat16) for _ in range(10)]
    qs = [torch.randn(26, 128, generator=g).to(torch.bfloat16) for _ in range(10)]
    om.score_chunk(qs, docs)
    t0, nm = time.time(), 0
    while nm == 0 or time.time() - t0 < seconds * 0.1:
        om.score_chunk(qs, docs)      # T2I chunk: 10 caption queries x 10 image docs
        om.score_chunk(docs, qs)      # I2T chunk: 10 image queries x 10 caption docs
        nm += 1
    tm = (time.time() - t0) / nm / 2
    calls = (n // 10) ** 2 + (n // 10) * (caps * n // 10)
    per_img = ti / ni + 6.0 * tc / nc + tm * calls / n
    return {"value": round(1.0 / per_img, 5), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/colpali_encoder.py bf16 CPU: {ni} images in {ti:.1f}s + {nc} queries (bs 4) in "
                      f"{tc:.1f}s, extrapolated to n images + 6n queries; + the reference's MaxSim chunk loop "
                      f"(oracle/maxsim.py) {tm * 1e3:.1f} ms per 10 x 10 chunk x {calls} calls",
            "maxsim_s": round(tm * calls, 2)}


def main_colpali(args, rank, world, dev):
    """BASELINE configs[3]: ColPali-v1.3, n images x 5n captions: encode (PaliGemma-3B) + MaxSim
    T2I / I2T / I2T-Sym + top-10 recall. value = images / job second."""
    from mme import get_spec, ops
    from mme.colpali_encoder import ColPaliModel
    from mme.distributed import all_reduce_, shard_range, sharded_colpali_recall
    spec = get_spec(args.model)
    model = ColPaliModel.from_spec(spec, seed=0, device=dev)
    n, caps = args.n_images, args.caps
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    imgs = torch.randint(0, 256, (n, 224, 224, 3), generator=g, device=dev, dtype=torch.uint8)
    all_caps = colpali_captions(n, caps)
    width = -(-max(len(spec.query_tokens(c)) for c in all_caps) // 16) * 16
    lo, hi = shard_range(n, rank, world)
    my_imgs = imgs[lo:hi].contiguous()
    my_caps = all_caps[caps * lo:caps * hi]
    my_t2i = my_caps[::caps]
    del imgs
    ev = {}
    last = {}

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev[name] = e

    def step():
        mark("t0")
        D = model.encode_images(my_imgs, batch=args.img_batch)
        dl = torch.full((D.shape[0],), D.shape[1], dtype=torch.int32, device=dev)
        Dp = torch.zeros(D.shape[0], -(-D.shape[1] // 16) * 16, D.shape[2], dtype=D.dtype, device=dev)
        Dp[:, : D.shape[1]] = D
        mark("img")
        Qt, qtl, qtp = model.encode_queries(my_t2i, exec_batch=args.txt_batch, width=width)
        Qa, qal, qap = model.encode_queries(my_caps, exec_batch=args.txt_batch, width=width)
        mark("txt")
        m, sc = sharded_colpali_recall(Dp, dl, Qt, qtl, Qa, qal, qap, rank, world, n, caps, return_scores=True)
        mark("score")
        last.update(tables=dict(D=Dp, dl=dl, Qt=Qt, qtl=qtl, qtp=qtp, Qa=Qa, qal=qal, qap=qap), scores=sc)
        return m

    if not args.no_kernel_timer:  # the warmup records into the timing-event pool, sizing it for the timed steps
        ops.KernelTimer.start()
    for _ in range(args.warmup):
        metrics = step()
    if not args.no_kernel_timer:
        ops.KernelTimer.stop()
        ops.KernelTimer.reserve(ops.KernelTimer.used() // max(args.warmup, 1) * args.steps + 64)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if not args.no_kernel_timer:
        ops.KernelTimer.start()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        metrics = step()
    barrier()
    dt = time.perf_counter() - t0
    ops.KernelTimer.stop()
    phases = {"encode_images_ms": ev["t0"].elapsed_time(ev["img"]), "encode_queries_ms": ev["img"].elapsed_time(ev["txt"]),
              "maxsim_recall_ms": ev["txt"].elapsed_time(ev["score"])}
    if world > 1:
        t = torch.tensor([dt], device=dev)
        all_reduce_(t, dist.ReduceOp.MAX)
        dt = float(t.item())
    kt = ops.KernelTimer.summary() if not args.no_kernel_timer else {}
    roofline = None
    if "gemm" in kt:
        gk = kt["gemm"]
        achieved = gk["flops"] / (gk["ms"] / 1e3) / 1e12
        roofline = {"bound": "mfma", "kernel": "mme_gemm (gemm_pipe9_kernel; gemm_pipe10_kernel for the non-split gelu_tanh / quick_gelu / gelu_erf fc1)", "achieved": round(achieved, 1),
                    "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4),
                    "traffic": None, "launches": gk["launches"], "avg_launch_ms": round(gk["ms"] / gk["launches"], 4),
                    "algorithmic_bytes_per_launch": round(gk["bytes"] / gk["launches"]),
                    "share_of_step_time": round(gk["ms"] / 1e3 / dt, 3)}
        if "attention" in kt:
            a = kt["attention"]
            roofline["attention_tflops"] = round(a["flops"] / (a["ms"] / 1e3) / 1e12, 1)
            roofline["attention_share"] = round(a["ms"] / 1e3 / dt, 3)
    value = n * args.steps / dt
    out = {
        "metric": "images/sec encode + end-to-end retrieval sec, 5k img x 25k cap; R@1 parity",
        "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": round(value / A40_COLPALI_IMG_S, 2) if args.model == "ColPali-v1.3" else None, "dtype": "bf16",
        "data": "synthetic (u8 224x224x3 images, token-id queries of 23-29 tokens; seeded random weights)",
        "config": {"workload": f"{args.model}: {n} images x {caps * n} captions (+{n} T2I), PaliGemma-3B encode + "
                               f"MaxSim T2I/I2T/Sym + top-10 recall", "n_images": n, "n_captions": caps * n,
                   "image_in": "224x224x3 u8", "image_size": spec.vision.image_size,
                   "image_tokens": len(spec.image_tokens), "img_batch": args.img_batch, "txt_batch": args.txt_batch,
                   "global_batch": n, "parallelism": f"image-shard x{world}"},
        "phases_rank0_last_step": {k: round(v, 1) for k, v in phases.items()},
        "recall": {k: round(v, 2) for k, v in metrics.items()},
        "roofline": roofline, "parity": None, "cpu_baseline": None,
    }
    out["process_group"] = ({"backend": dist.get_backend(), "ranks": dist.get_world_size(),
                             "same_device": bool(args.same_device)} if world > 1 else None)
    if rank == 0 and world == 1 and not args.no_parity:
        out["parity"] = colpali_parity(last["tables"], last["scores"], caps, imgs_u8=my_imgs, t2i_caps=my_t2i)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        out["cpu_baseline"] = cpu_baseline_colpali(spec, args.cpu_seconds, n, caps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    from mme import launch
    if args.gpus is None and not launch.under_launcher():
        args.gpus = 1
    if args.gpus is not None and args.gpus > 1 and not launch.under_launcher():
        # `python bench.py --gpus N` without torchrun: start N rank processes of this script
        # BEFORE anything touches the GPU (this parent never initialises HIP), and exit with
        # the first failing rank's status
        sys.exit(launch.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    if args.gemm_form is not None or args.attn_form is not None or args.mx_form is not None:  # thread-local forms
        import contextlib
        from mme import ops as _ops
        _forms = contextlib.ExitStack()
        _forms.enter_context(_ops.kernel_forms(**({"gemm": args.gemm_form} if args.gemm_form is not None else {}),
                                               **({"attention_long": args.attn_form} if args.attn_form is not None else {}),
                                               **({"mx": args.mx_form} if args.mx_form is not None else {})))
    _, _, local = launch.env_rank_world()
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    try:
        rank, world, _ = launch.init_distributed(args.gpus, args.backend, dev, same_device=args.same_device)
    except launch.LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(3)
    if args.model.startswith("ColPali"):
        if args.n_images is None:
            args.n_images = 1000  # BASELINE configs[3]: 1 000 images x 5 000 captions
        if args.img_batch is None:
            args.img_batch = 32
        if args.txt_batch is None:
            args.txt_batch = 2048
        return main_colpali(args, rank, world, dev)

    from mme import get_spec, ops
    from mme.distributed import all_reduce_, shard_range, sharded_recall
    from mme.models import load_model

    spec = get_spec(args.model)
    if args.n_images is None:
        args.n_images = 5000  # BASELINE configs[1], [2], [4]: 5 000 images x 25 000 captions
    eb_img, eb_txt = exec_batches(spec)
    args.img_batch = eb_img if args.img_batch is None else args.img_batch
    args.txt_batch = eb_txt if args.txt_batch is None else args.txt_batch
    model, _ = load_model(args.model, seed=0, device=dev, fp8=args.fp8)
    n, caps = args.n_images, args.caps
    imgs, ids = synth_inputs(spec, n, caps, dev)
    lo, hi = shard_range(n, rank, world)
    my_imgs = imgs[lo:hi].contiguous()
    my_caps = ids[caps * lo:caps * hi].contiguous()
    my_t2i = my_caps[::caps].contiguous()
    del imgs, ids
    torch.cuda.synchronize()
    # encoder parity items: the first, middle and last images / T2I captions of this rank's job, i.e.
    # rows at both ends of different execution batches (7 items, ~7 s of fp32 CPU work for SigLIP-400M)
    nl = my_imgs.shape[0]
    enc_idx = sorted({i for i in (0, 1, nl // 4, nl // 2, 3 * nl // 4, nl - 2, nl - 1) if 0 <= i < nl})
    n_enc = len(enc_idx)

    last = {}
    ev = {}

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev[name] = e

    def step():
        mark("t0")
        img = model.encode_images(my_imgs, batch=args.img_batch)
        mark("img")
        t2i = model.encode_texts(my_t2i, exec_batch=args.txt_batch)
        allc = model.encode_texts(my_caps, exec_batch=args.txt_batch)
        mark("txt")
        m, tables = sharded_recall(img, t2i, allc, rank, world, n, caps, return_tables=True)
        mark("ret")
        last.update(img=img, t2i=t2i, allc=allc, tables=tables)
        return m

    if not args.no_kernel_timer:  # the warmup records into the timing-event pool, sizing it for the timed steps
        ops.KernelTimer.start()
    for _ in range(args.warmup):
        metrics = step()
    if not args.no_kernel_timer:
        ops.KernelTimer.stop()
        ops.KernelTimer.reserve(ops.KernelTimer.used() // max(args.warmup, 1) * args.steps + 64)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    if not args.no_kernel_timer:
        ops.KernelTimer.start()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        metrics = step()
    barrier()
    dt = time.perf_counter() - t0
    ops.KernelTimer.stop()
    # phases of the last timed step (device events on the launch stream), max over ranks
    phases = torch.tensor([ev["t0"].elapsed_time(ev["img"]), ev["img"].elapsed_time(ev["txt"]),
                           ev["txt"].elapsed_time(ev["ret"])], dtype=torch.float64, device=dev)
    gev = last["tables"].get("gather_events")
    gather_ms = gev[0].elapsed_time(gev[1]) if gev is not None else 0.0
    allgather_per_rank = [round(gather_ms / 1e3, 5)]
    # per-rank record of the last timed step (so an N-GPU line names the rank / phase that limits it):
    # phases (s), this rank's image count, its wall time of the K timed steps (s), the all-gather (s)
    per_rank = torch.zeros(world, 7, dtype=torch.float64, device=dev)
    per_rank[rank] = torch.tensor([phases[0] / 1e3, phases[1] / 1e3, phases[2] / 1e3, hi - lo, my_caps.shape[0],
                                   dt, gather_ms / 1e3], dtype=torch.float64)
    if world > 1:
        t = torch.tensor([dt], device=dev)
        all_reduce_(t, dist.ReduceOp.MAX)
        dt = float(t.item())
        all_reduce_(phases, dist.ReduceOp.MAX)
        all_reduce_(per_rank, dist.ReduceOp.SUM)
        allgather_per_rank = [round(x, 5) for x in per_rank[:, 6].tolist()]
    phases = phases.tolist()
    pr = per_rank.tolist()
    per_rank_line = {"encode_images_s": [round(r[0], 4) for r in pr], "encode_texts_s": [round(r[1], 4) for r in pr],
                     "retrieval_s": [round(r[2], 4) for r in pr], "n_images": [int(r[3]) for r in pr],
                     "n_captions": [int(r[4]) for r in pr], "timed_s": [round(r[5], 4) for r in pr],
                     "slowest_rank": max(range(world), key=lambda i: pr[i][0] + pr[i][1] + pr[i][2])}
    kt = ops.KernelTimer.summary() if not args.no_kernel_timer else {}

    roofline = None
    fam = "gemm_mx" if args.fp8 else "gemm"
    if fam in kt:
        # dominant kernel family: mme_gemm (gemm_pipe9_kernel; gemm_pipe6_kernel where K % 64 != 0;
        # gemm_tn_kernel for the few small shapes),
        # or with --fp8 mme_gemm_mx (gemm_mx11_kernel since round 4, block-scaled fp8 MFMA; dense fp8 peak).
        # achieved = algorithmic FLOPs per launch (2*M*N*K, zero-padding excluded) / average launch time
        # from HIP events recorded on the launch stream over the timed region.
        g = kt[fam]
        avg_ms = g["ms"] / g["launches"]
        achieved = g["flops"] / (g["ms"] / 1e3) / 1e12
        peak = MFMA_FP8_PEAK_TFLOPS if args.fp8 else MFMA_BF16_PEAK_TFLOPS
        roofline = {"bound": "mfma",
                    "kernel": "mme_gemm_mx (gemm_mx11_kernel)" if args.fp8 else "mme_gemm (gemm_pipe9_kernel; gemm_pipe10_kernel for the non-split gelu_tanh / quick_gelu / gelu_erf fc1)",
                    "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                    "traffic": None, "launches": g["launches"], "avg_launch_ms": round(avg_ms, 4),
                    "algorithmic_bytes_per_launch": round(g["bytes"] / g["launches"]),
                    "share_of_step_time": round(g["ms"] / 1e3 / dt, 3)}
        if args.fp8 and "gemm" in kt:
            b = kt["gemm"]
            roofline["bf16_gemm_tflops"] = round(b["flops"] / (b["ms"] / 1e3) / 1e12, 1)
            roofline["bf16_gemm_share"] = round(b["ms"] / 1e3 / dt, 3)
        # HBM bytes per launch from the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_gemm.sh,
        # gfx950-corrected by tools/pmc_summary.py) over one job of THIS geometry: used only when the pass
        # saw the same GEMM launch count per job as this run's timed steps (same batches, same mix)
        pmc = load_traffic(args.model, n, args.img_batch, args.txt_batch, args.fp8)
        per_job = g["launches"] // max(args.steps, 1)
        pl = pmc.get(fam, {}).get("launches", 0) if pmc else 0
        # the PMC job also holds the model load's few GEMMs (one MAP-head preparation launch): the same
        # launch mix when the counts agree within 0.5 %
        if pmc and abs(pl - per_job) <= 0.005 * per_job:
            roofline["traffic"] = round(pmc[fam]["hbm_bytes_per_launch"])
            roofline["traffic_source"] = pmc["_source"] + f", {pl} launches per job vs {per_job} timed"
        elif pmc:
            roofline["traffic_note"] = (f"{pmc['_source']} holds {pmc.get(fam, {}).get('launches')} {fam} launches "
                                        f"per job, this run {per_job}: not the same launch mix, not reported")
        if "attention" in kt:
            a = kt["attention"]
            roofline["attention_tflops"] = round(a["flops"] / (a["ms"] / 1e3) / 1e12, 1)
            roofline["attention_share"] = round(a["ms"] / 1e3 / dt, 3)
        roofline["hbm_kernels"] = hbm_rooflines(kt, dt, pmc, args.steps)

    value = n * args.steps / dt
    out = {
        "metric": "images/sec encode + end-to-end retrieval sec, 5k img x 25k cap; R@1 parity",
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "strong",  # total job fixed (5k images) as N grows
        "vs_baseline": round(value / A40_PUBLISHED_IMG_S, 2) if (args.model == "SigLIP-400M" and n == 5000) else None,
        "dtype": "mx-fp8 (e4m3 + e8m0/32) QKV/MLP GEMMs, bf16 elsewhere" if args.fp8 else "bf16",
        "data": "synthetic (u8 224x224x3 images, token-id captions L=%d; seeded random weights)" % spec.text.max_pos,
        "config": {"workload": f"{args.model}: {n} images x {caps * n} captions (+{n} T2I), encode + sim + top-10 "
                               f"recall", "n_images": n, "n_captions": caps * n, "image_in": "224x224x3 u8",
                   "image_size": spec.vision.image_size, "seq_len": spec.text.max_pos, "img_batch": args.img_batch,
                   "txt_batch": args.txt_batch, "global_batch": n, "parallelism": f"image-shard x{world}",
                   **({"gemm_form": args.gemm_form} if args.gemm_form is not None else {}),
                   **({"attn_form": args.attn_form} if args.attn_form is not None else {}),
                   **({"mx_form": args.mx_form} if args.mx_form is not None else {})},
        "recall": {k: round(v, 2) for k, v in metrics.items()},
        # last timed step, device events, max over ranks; retrieval = all-gather (N > 1) + T2I / I2T /
        # I2T-Sym similarity + fused top-10 + recall counters + counter all-reduce
        "encode_images_s": round(phases[0] / 1e3, 4), "encode_texts_s": round(phases[1] / 1e3, 4),
        "retrieval_s": round(phases[2] / 1e3, 4),
        # per rank, last timed step: the RCCL all-gathers of the image / T2I / caption tables
        # (device events around them; 0 at N = 1 where nothing is gathered)
        "allgather_s_per_rank": allgather_per_rank,
        # the same phases per rank (index = rank), with each rank's share and its own timed wall clock
        "per_rank": per_rank_line,
        "roofline": roofline,
        "parity": None,
        "cpu_baseline": None,
    }
    out["process_group"] = ({"backend": dist.get_backend(), "ranks": dist.get_world_size(),
                             "same_device": bool(args.same_device)} if world > 1 else None)
    if rank == 0 and not args.no_parity:
        out["parity"] = retrieval_parity(last["tables"], metrics, caps)
        if n_enc:
            ii = torch.tensor(enc_idx, device=my_imgs.device)
            out["parity"]["encoders"] = encoder_parity(spec, my_imgs[ii], my_t2i[ii], last["img"][ii], last["t2i"][ii],
                                                       bar=0.99 if args.fp8 else 0.999)
            out["parity"]["encoders"]["rows"] = enc_idx
        if args.fp8 and world == 1:
            out["fp8_drift"] = fp8_drift(args.model, dev, my_imgs, my_t2i, my_caps, last["tables"], args.img_batch,
                                         args.txt_batch, caps)
    if args.host_inputs:
        host_imgs = my_imgs.cpu().pin_memory()
        barrier()
        th = time.perf_counter()
        img = model.encode_images(host_imgs, batch=args.img_batch)
        t2i = model.encode_texts(my_t2i, exec_batch=args.txt_batch)
        allc = model.encode_texts(my_caps, exec_batch=args.txt_batch)
        sharded_recall(img, t2i, allc, rank, world, n, caps)
        barrier()
        out["host_inputs_img_s"] = round(n / (time.perf_counter() - th), 2)
    if world == 1 and args.bootstrap > 0:
        from mme import bootstrap as mb
        torch.cuda.synchronize()
        tb = time.perf_counter()
        s_t2i, s_i2t = mb.full_scores(last["img"], last["t2i"], last["allc"])
        hits = mb.bootstrap_hits(s_t2i, s_i2t, mb.sample_indices(n, args.bootstrap, seed=0, device=dev), caps)
        torch.cuda.synchronize()
        tb = time.perf_counter() - tb
        row = mb.bootstrap_row(hits, n)
        out["bootstrap"] = {"iterations": args.bootstrap, "seconds": round(tb, 3),
                            "T2I_R@1_mean": round(row["T2I_R@1_mean"], 3),
                            "T2I_R@1_ci95": [round(row["T2I_R@1_lower"], 3), round(row["T2I_R@1_upper"], 3)],
                            "note": "full score matrices once + per-resample gather/top-10/recall on the device"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        out["cpu_baseline"] = cpu_baseline(spec, args.cpu_seconds, last["tables"], caps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
