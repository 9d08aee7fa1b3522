#!/usr/bin/env python3
"""Preprocess (PIL-bicubic resize + crop + normalise + im2col) timing at the bench's shapes.

Algorithmic bytes per image: the u8 source raster read once + the bf16 im2col rows written
(G*G x kpad). Prints ms per call and TB/s; HIP events on the launch stream.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mme import ops  # noqa: E402
from mme.config import IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD  # noqa: E402

CASES = {  # name: (n, H, W, S, patch, kpad)
    "siglip384": (239, 224, 224, 384, 14, 640),
    "dfn5b378": (128, 224, 224, 378, 14, 640),
    "clip336": (256, 224, 224, 336, 14, 640),
    "vith224": (256, 224, 224, 224, 14, 640),
    "colpali448": (32, 224, 224, 448, 14, 592),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cases", default=",".join(CASES))
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    res = {}
    for name in a.cases.split(","):
        n, H, W, S, patch, kpad = CASES[name]
        x = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (n, H, W, 3), dtype=np.uint8)).cuda()
        kw = dict(resize=(S, S), crop=(0, 0), size=S, mean=IMAGENET_STANDARD_MEAN, std=IMAGENET_STANDARD_STD,
                  patch=patch, kpad=kpad)
        out = ops.preprocess_u8(x, **kw)
        for _ in range(3):
            ops.preprocess_u8(x, **kw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ms = 1e30
        for _ in range(3):
            s.record()
            for _ in range(a.iters):
                ops.preprocess_u8(x, **kw)
            e.record()
            torch.cuda.synchronize()
            ms = min(ms, s.elapsed_time(e) / a.iters)
        G = S // patch
        nbytes = n * (H * W * 3 + G * G * kpad * 2)
        res[name] = {"ms": round(ms, 4), "tb_s": round(nbytes / ms / 1e9, 3), "bytes": nbytes}
        print(f"{name:11s} n={n} {H}x{W} -> {S} p{patch}: {ms:7.3f} ms  {nbytes / ms / 1e9:6.2f} TB/s "
              f"({nbytes / 1e6:.1f} MB)", flush=True)
        del out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
