"""Validate the bench's CPU baseline stand-in against the reference itself (run in the dev container).

bench.py's cpu_baseline times oracle/encoders.py (the build's bf16 PyTorch-CPU restatement)
on the GPU box, where the reference cannot travel. SURVEY §8d asks for the stand-in to be
timed side by side with the reference's own main.encode_data (main.py:386-438) in this
container at the reference's batch size 32, with a ratio of about 1. This script does that
on the SAME inputs and weights (SigLIP-400M full architecture, deterministic random weights,
bf16, torch threads = all cores) and writes profiles/r02_cpu_baseline_check.json.

    python tools/cpu_baseline_check.py [--model SigLIP-400M] [--images 32] [--captions 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="SigLIP-400M")
    ap.add_argument("--images", type=int, default=32)
    ap.add_argument("--captions", type=int, default=64)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_baseline_check.json"))
    args = ap.parse_args()
    from PIL import Image
    import make_goldens as mg
    from mme.config import get_spec
    from mme.processor import synthetic_caption_ids, synthetic_images
    from oracle import encoders as oe
    from weights_gen import torch_state_dict
    main = mg.import_reference()
    spec = get_spec(args.model)
    threads = os.cpu_count()
    torch.set_num_threads(threads)
    imgs = synthetic_images(args.images)
    caps = synthetic_caption_ids(spec, args.captions).tolist()
    S = spec.vision.image_size
    if spec.family == "siglip":
        from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
        ip = SiglipImageProcessorPil(size={"height": S, "width": S})
    else:
        from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil
        ip = CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S})
    proc = mg.RefProcessor(ip, spec.text.pad_id)
    m_info = {"name": args.model, "type": spec.m_info["type"], "batch_size": 32}
    res = {"model": args.model, "threads": threads, "batch_size": 32, "images": args.images,
           "captions": args.captions, "dtype": "bf16"}

    # the reference: main.encode_data over the transformers modules (what main.py loads)
    hf = mg.RefAdapter(mg.hf_model(spec, torch.bfloat16))
    main.DEVICE, main.DTYPE = "cpu", torch.bfloat16
    pil = [Image.fromarray(a) for a in imgs]
    with torch.no_grad():
        main.encode_data(hf, proc, m_info, pil[:1], caps[:1])  # warm-up
        t0 = time.time()
        ri, _ = main.encode_data(hf, proc, m_info, pil, [])
        t1 = time.time()
        _, rt = main.encode_data(hf, proc, m_info, [], caps)
        t2 = time.time()
    res["reference"] = {"img_s": args.images / (t1 - t0), "cap_s": args.captions / (t2 - t1),
                        "what": "main.encode_data (HF SiglipModel/CLIPModel + PIL image processor), bf16"}
    del hf

    # the stand-in: oracle/encoders.py (bf16 PyTorch-CPU restatement, numpy PIL-exact preprocessing)
    sd = torch_state_dict(spec, 0, torch.bfloat16)
    oe.encode_data(spec, sd, list(imgs[:1]), caps[:1], bs=1)
    t0 = time.time()
    oi, _ = oe.encode_data(spec, sd, list(imgs), [], bs=32)
    t1 = time.time()
    _, ot = oe.encode_data(spec, sd, [], caps, bs=32)
    t2 = time.time()
    res["oracle"] = {"img_s": args.images / (t1 - t0), "cap_s": args.captions / (t2 - t1),
                     "what": "oracle/encoders.py encode_data, bf16"}
    for side in ("reference", "oracle"):
        r = res[side]
        r["job_img_per_s"] = 1.0 / (1.0 / r["img_s"] + 6.0 / r["cap_s"])  # n images + 6n captions
        for k in list(r):
            if isinstance(r[k], float):
                r[k] = round(r[k], 4)
    res["ratio_oracle_over_reference"] = {k: round(res["oracle"][k] / res["reference"][k], 3)
                                          for k in ("img_s", "cap_s", "job_img_per_s")}
    cos_i = torch.nn.functional.cosine_similarity(oi.float(), ri.float()).min().item()
    cos_t = torch.nn.functional.cosine_similarity(ot.float(), rt.float()).min().item()
    res["embedding_cos_min"] = {"images": round(cos_i, 5), "captions": round(cos_t, 5)}
    res["host"] = os.uname().nodename
    print(json.dumps(res, indent=1))
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
