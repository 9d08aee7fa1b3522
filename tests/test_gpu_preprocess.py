"""Device preprocessing vs PIL + HF (tests/golden/preprocess.npz): bit-exact."""
import numpy as np
import pytest
import torch

from mme import ops
from mme.config import IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD, OPENAI_CLIP_MEAN, OPENAI_CLIP_STD, ImageProcConfig
from mme.processor import image_geometry
from oracle import pil_bicubic

pytestmark = pytest.mark.gpu
CASES = ["siglip384", "clip336", "dfn378", "clip336_nonsq", "vith224_down"]


def _cfg(kind, S):
    if kind == 0:
        return ImageProcConfig(S, "square", IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD)
    return ImageProcConfig(S, "shortest_edge", OPENAI_CLIP_MEAN, OPENAI_CLIP_STD)


@pytest.mark.parametrize("case", CASES)
def test_preprocess_pixel_values_bit_exact(cuda, golden, case):
    g = golden("preprocess")
    H, W, S, kind = (int(v) for v in g[case + "_meta"])
    ip = _cfg(kind, S)
    rh, rw, top, left = image_geometry(H, W, ip)
    imgs = torch.from_numpy(g[case + "_in"][None]).cuda()
    pv = ops.preprocess_u8(imgs, resize=(rh, rw), crop=(top, left), size=S, mean=ip.mean, std=ip.std)
    ref = pil_bicubic.normalize(g[case + "_u8"], ip.mean, ip.std)
    got = pv[0].cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), \
        f"{case}: {np.sum(got != ref)} pixel values differ from PIL+HF"


# patches: the fused kernel (one workgroup per patch row, LDS-staged rows) at every golden
# geometry (S % 14 != 0 for SigLIP 384 and DFN5B 378: the last pixels feed no patch)
@pytest.mark.parametrize("case", CASES)
def test_preprocess_patches_match_im2col(cuda, golden, case):
    g = golden("preprocess")
    H, W, S, kind = (int(v) for v in g[case + "_meta"])
    ip = _cfg(kind, S)
    rh, rw, top, left = image_geometry(H, W, ip)
    imgs = torch.from_numpy(np.stack([g[case + "_in"]] * 3)).cuda()
    patches = ops.preprocess_u8(imgs, resize=(rh, rw), crop=(top, left), size=S, mean=ip.mean, std=ip.std,
                                patch=14, kpad=640)
    pv = torch.from_numpy(pil_bicubic.normalize(g[case + "_u8"], ip.mean, ip.std)).cuda()
    ref = ops.im2col(pv[None].expand(3, -1, -1, -1).contiguous(), 14, 640)
    assert torch.equal(patches, ref)


def test_preprocess_batch_of_synthetic(cuda):
    rng = np.random.default_rng(11)
    imgs = rng.integers(0, 256, (6, 224, 224, 3), dtype=np.uint8)
    ip = _cfg(0, 384)
    pv = ops.preprocess_u8(torch.from_numpy(imgs).cuda(), resize=(384, 384), crop=(0, 0), size=384, mean=ip.mean,
                           std=ip.std).cpu().numpy()
    for i in range(6):
        ref = pil_bicubic.normalize(pil_bicubic.preprocess_u8(imgs[i], 384, "square"), ip.mean, ip.std)
        assert np.array_equal(pv[i], ref)


def test_preprocess_patches_large_downscale_fallback(cuda):
    """A 1500 x 1300 image to 224 (CLIP shortest edge + crop): a patch row needs more input rows
    than the fused kernel stages in LDS, so the two-kernel path runs; both equal im2col of the
    bit-exact pixel values."""
    rng = np.random.default_rng(3)
    imgs = rng.integers(0, 256, (2, 1500, 1300, 3), dtype=np.uint8)
    ip = _cfg(1, 224)
    rh, rw, top, left = image_geometry(1500, 1300, ip)
    x = torch.from_numpy(imgs).cuda()
    patches = ops.preprocess_u8(x, resize=(rh, rw), crop=(top, left), size=224, mean=ip.mean, std=ip.std,
                                patch=14, kpad=640)
    pv = ops.preprocess_u8(x, resize=(rh, rw), crop=(top, left), size=224, mean=ip.mean, std=ip.std)
    assert torch.equal(patches, ops.im2col(pv, 14, 640))
    ref = pil_bicubic.normalize(pil_bicubic.preprocess_u8(imgs[1], 224, "shortest_edge"), ip.mean, ip.std)
    assert np.array_equal(pv[1].cpu().numpy(), ref)


def test_preprocess_patches_batch_vs_pixel_values(cuda):
    """The production batch shape (SigLIP 384, 40 images): fused patches == im2col(pixel_values)."""
    rng = np.random.default_rng(12)
    x = torch.from_numpy(rng.integers(0, 256, (40, 224, 224, 3), dtype=np.uint8)).cuda()
    ip = _cfg(0, 384)
    kw = dict(resize=(384, 384), crop=(0, 0), size=384, mean=ip.mean, std=ip.std)
    patches = ops.preprocess_u8(x, patch=14, kpad=640, **kw)
    assert torch.equal(patches, ops.im2col(ops.preprocess_u8(x, **kw), 14, 640))


# round 3: p = 14 runs resample_patch_p_kernel<14> (compile-time patch, <= 8 taps per pass);
# other patch sizes and wider filters the generic fused kernel. Both == im2col of the bit-exact
# pixel values, upscales and mild downscales (448 -> 384: 7 taps), ragged S % p.
@pytest.mark.parametrize("H,W,S,patch,kpad", [(224, 224, 384, 14, 640), (448, 448, 384, 14, 640),
                                              (300, 500, 378, 14, 640), (224, 224, 384, 16, 768),
                                              (256, 256, 224, 16, 768), (224, 224, 448, 14, 592)])
def test_preprocess_patch_kernels_vs_pixel_values(cuda, H, W, S, patch, kpad):
    rng = np.random.default_rng(H + W + S + patch)
    x = torch.from_numpy(rng.integers(0, 256, (5, H, W, 3), dtype=np.uint8)).cuda()
    ip = _cfg(0, S)
    kw = dict(resize=(S, S), crop=(0, 0), size=S, mean=ip.mean, std=ip.std)
    patches = ops.preprocess_u8(x, patch=patch, kpad=kpad, **kw)
    assert torch.equal(patches, ops.im2col(ops.preprocess_u8(x, **kw), patch, kpad))
