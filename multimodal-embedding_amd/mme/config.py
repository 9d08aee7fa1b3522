"""Model registry: the dense dual encoders of the reference's model table.

The reference loads these by hub id (main.py:127-142, 808-820); offline, the
architecture constants below (public HF configs, confirmed by parameter count
in SURVEY.md §6) are instantiated with seeded random weights or with a local
safetensors / HF state dict (mme.weights).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, Optional, Sequence, Tuple

from ._lib import ACT_GELU_ERF, ACT_GELU_TANH, ACT_QUICK_GELU

OPENAI_CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_CLIP_STD = (0.26862954, 0.26130258, 0.27577711)
# Execution batches of the dense jobs (images / captions per tower launch sequence; tail_aware_batch
# then picks equal splits): 512 / 4096 (SigLIP 512 / 8192) since round 3 -- SigLIP-400M's 5k x 25k job runs 12 x 417
# images and 5 x 5 000 (+ 1 x 5 000 T2I) captions: 512 / 4096 gained +0.5-1.0 % over 256 / 2048
# (239 / 1 563; fewer launches and fill / drain edges; profiles/r03_v20_batch_sweep.log), 8192
# captions another -1 % of SigLIP's text tower time (profiles/r03_v28_txt_batch_8192.log) but +1.6 %
# on LAION-CLIP-H's (level on CLIP-L; profiles/r03_v29_clip_txt_batch_8192.log), so the 8192 cap is
# SigLIP's only. bench.py's defaults and the tests' production geometry (tests/test_gpu_encoders.py)
# read exec_batches().
EXEC_IMG_BATCH = 512
EXEC_TXT_BATCH = 4096
EXEC_TXT_BATCH_SIGLIP = 8192

IMAGENET_STANDARD_MEAN = (0.5, 0.5, 0.5)
IMAGENET_STANDARD_STD = (0.5, 0.5, 0.5)

ACTS = {"gelu_pytorch_tanh": ACT_GELU_TANH, "quick_gelu": ACT_QUICK_GELU, "gelu": ACT_GELU_ERF}


@dataclass(frozen=True)
class TowerConfig:
    hidden: int
    intermediate: int
    layers: int
    heads: int
    act: str
    eps: float

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    @property
    def inter_pad(self) -> int:
        """Intermediate width padded to a multiple of 128 (zero rows/cols; gelu(0) = 0)."""
        return (self.intermediate + 127) // 128 * 128


@dataclass(frozen=True)
class VisionConfig(TowerConfig):
    image_size: int = 224
    patch: int = 14

    @property
    def grid(self) -> int:
        return self.image_size // self.patch

    @property
    def num_patches(self) -> int:
        return self.grid ** 2

    @property
    def kpad(self) -> int:
        """Patch-embedding GEMM K (3*p*p) padded to a multiple of 64."""
        return (3 * self.patch * self.patch + 63) // 64 * 64


@dataclass(frozen=True)
class TextConfig(TowerConfig):
    vocab: int = 49408
    max_pos: int = 77
    eos_id: int = 49407
    bos_id: Optional[int] = 49406
    pad_id: int = 49407
    pool: str = "eos"  # "eos" (first eos), "argmax" (legacy eos_token_id == 2), "last" (SigLIP)
    causal: bool = True


@dataclass(frozen=True)
class ImageProcConfig:
    size: int                      # final (cropped) size S
    mode: str                      # "square" (SigLIP: resize to S x S) | "shortest_edge" (CLIP: resize + center crop)
    mean: Tuple[float, float, float]
    std: Tuple[float, float, float]


@dataclass(frozen=True)
class ModelSpec:
    name: str
    hub_id: str
    family: str                    # "siglip" | "clip"
    vision: VisionConfig
    text: TextConfig
    proj_dim: int                  # joint embedding width D
    image_proc: ImageProcConfig
    batch_size: int = 32           # main.py:131-136 (ARGS.batch_size default 32, main.py:73)
    extra: Dict[str, str] = field(default_factory=dict)

    @property
    def m_info(self) -> dict:
        """The reference's m_info dict (main.py:130-136)."""
        typ = "siglip" if self.family == "siglip" else "dense"
        return {"name": self.name, "id": self.hub_id, "type": typ, "batch_size": self.batch_size}

    def with_batch_size(self, bs: int) -> "ModelSpec":
        return replace(self, batch_size=bs)


def _siglip_400m() -> ModelSpec:
    v = VisionConfig(hidden=1152, intermediate=4304, layers=27, heads=16, act="gelu_pytorch_tanh", eps=1e-6,
                     image_size=384, patch=14)
    t = TextConfig(hidden=1152, intermediate=4304, layers=27, heads=16, act="gelu_pytorch_tanh", eps=1e-6,
                   vocab=32000, max_pos=64, eos_id=1, bos_id=None, pad_id=1, pool="last", causal=False)
    return ModelSpec("SigLIP-400M", "google/siglip-so400m-patch14-384", "siglip", v, t, 1152,
                     ImageProcConfig(384, "square", IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD))


def _clip(name, hub, v_hidden, v_inter, v_layers, image_size, v_act, t_hidden, t_inter, t_layers, t_heads, t_act,
          proj, pool="eos") -> ModelSpec:
    v = VisionConfig(hidden=v_hidden, intermediate=v_inter, layers=v_layers, heads=16, act=v_act, eps=1e-5,
                     image_size=image_size, patch=14)
    t = TextConfig(hidden=t_hidden, intermediate=t_inter, layers=t_layers, heads=t_heads, act=t_act, eps=1e-5,
                   pool=pool)
    return ModelSpec(name, hub, "clip", v, t, proj,
                     ImageProcConfig(image_size, "shortest_edge", OPENAI_CLIP_MEAN, OPENAI_CLIP_STD))


REGISTRY: Dict[str, ModelSpec] = {
    "SigLIP-400M": _siglip_400m(),
    # openai config.json keeps the legacy text eos_token_id == 2 -> argmax pooling (TF:…clip.py:561-570)
    "OpenAI-CLIP-L": _clip("OpenAI-CLIP-L", "openai/clip-vit-large-patch14-336", 1024, 4096, 24, 336, "quick_gelu",
                           768, 3072, 12, 12, "quick_gelu", 768, pool="argmax"),
    "LAION-CLIP-H": _clip("LAION-CLIP-H", "laion/CLIP-ViT-H-14-laion2B-s32B-b79K", 1280, 5120, 32, 224, "gelu",
                          1024, 4096, 24, 16, "gelu", 1024),
    "MetaCLIP-H14": _clip("MetaCLIP-H14", "facebook/metaclip-h14-fullcc2.5b", 1280, 5120, 32, 224, "quick_gelu",
                          1024, 4096, 24, 16, "quick_gelu", 1024),
    "Apple-DFN5B-H": _clip("Apple-DFN5B-H", "apple/DFN5B-CLIP-ViT-H-14-378", 1280, 5120, 32, 378, "quick_gelu",
                           1024, 4096, 24, 16, "quick_gelu", 1024),
}

# Small configurations with the same code paths (head dims 72 / 80 / 64, ragged
# token counts, padded intermediate widths) for parity tests.
TINY: Dict[str, ModelSpec] = {
    "tiny-siglip": ModelSpec(
        "tiny-siglip", "-", "siglip",
        VisionConfig(hidden=576, intermediate=600, layers=2, heads=8, act="gelu_pytorch_tanh", eps=1e-6,
                     image_size=98, patch=14),
        TextConfig(hidden=576, intermediate=600, layers=2, heads=8, act="gelu_pytorch_tanh", eps=1e-6, vocab=1000,
                   max_pos=16, eos_id=1, bos_id=None, pad_id=1, pool="last", causal=False),
        576, ImageProcConfig(98, "square", IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD), batch_size=4),
    "tiny-clip": ModelSpec(
        "tiny-clip", "-", "clip",
        VisionConfig(hidden=320, intermediate=640, layers=2, heads=4, act="quick_gelu", eps=1e-5, image_size=56,
                     patch=14),
        TextConfig(hidden=256, intermediate=512, layers=2, heads=4, act="gelu", eps=1e-5, vocab=1000, max_pos=20,
                   eos_id=999, bos_id=998, pad_id=999, pool="eos", causal=True),
        256, ImageProcConfig(56, "shortest_edge", OPENAI_CLIP_MEAN, OPENAI_CLIP_STD), batch_size=4),
}


@dataclass(frozen=True)
class GemmaConfig:
    """Gemma decoder of PaliGemma (TF:models/gemma/configuration_gemma.py:64-83)."""
    hidden: int
    intermediate: int
    layers: int
    heads: int            # query heads; ONE key/value head (MQA)
    head_dim: int
    vocab: int
    eps: float = 1e-6
    theta: float = 10000.0


@dataclass(frozen=True)
class ColPaliSpec:
    """ColPali = PaliGemma (SigLIP vision tower without head + Gemma) + 128-d head.

    Token layout (TF:models/colpali/processing_colpali.py:113-142): an image is
    [<image>] * P + [bos] + prompt("Describe the image.") + ["\\n"]; a query is
    [bos] + prefix("Question: ") + caption + [pad] * 10 (query augmentation) + ["\\n"].
    The Gemma tokenizer pads on the LEFT (TF:models/gemma/tokenization_gemma.py:55).
    Vocab files are absent offline: prompt / prefix ids are fixed synthetic ids."""
    name: str
    hub_id: str
    vision: VisionConfig
    text: GemmaConfig
    image_proc: ImageProcConfig
    image_token_id: int
    bos_id: int = 2
    eos_id: int = 1
    pad_id: int = 0
    newline_id: int = 108
    prompt_ids: Tuple[int, ...] = (50721, 573, 2416, 235265)   # synthetic "Describe the image."
    query_prefix_ids: Tuple[int, ...] = (9413, 235292, 235248)  # synthetic "Question: "
    query_prefix: str = "Question: "   # the text layout of string queries (ColPaliProcessor.query_prefix)
    n_aug: int = 10
    dim: int = 128
    batch_size: int = 4   # main.py:130
    family: str = "colpali"

    @property
    def image_seq_len(self) -> int:
        return self.vision.num_patches

    @property
    def image_tokens(self) -> Tuple[int, ...]:
        return (self.image_token_id,) * self.image_seq_len + (self.bos_id,) + self.prompt_ids + (self.newline_id,)

    def query_tokens(self, caption: Sequence[int]) -> Tuple[int, ...]:
        return ((self.bos_id,) + self.query_prefix_ids + tuple(int(c) for c in caption) +
                (self.pad_id,) * self.n_aug + (self.newline_id,))

    @property
    def m_info(self) -> dict:
        return {"name": self.name, "id": self.hub_id, "type": "colpali", "batch_size": self.batch_size}

    def with_batch_size(self, bs: int) -> "ColPaliSpec":
        return replace(self, batch_size=bs)


COLPALI: Dict[str, ColPaliSpec] = {
    # vidore/colpali-v1.3 on PaliGemma-3B-pt-448 (vision 27 x 1152, Gemma-2B 18 x 2048, MQA 8 x 256)
    "ColPali-v1.3": ColPaliSpec(
        "ColPali-v1.3", "vidore/colpali-v1.3",
        VisionConfig(hidden=1152, intermediate=4304, layers=27, heads=16, act="gelu_pytorch_tanh", eps=1e-6,
                     image_size=448, patch=14),
        GemmaConfig(hidden=2048, intermediate=16384, layers=18, heads=8, head_dim=256, vocab=257216),
        ImageProcConfig(448, "square", IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD), image_token_id=257152),
    "tiny-colpali": ColPaliSpec(
        "tiny-colpali", "-",
        VisionConfig(hidden=576, intermediate=600, layers=2, heads=8, act="gelu_pytorch_tanh", eps=1e-6,
                     image_size=56, patch=14),
        GemmaConfig(hidden=512, intermediate=1024, layers=2, heads=2, head_dim=256, vocab=1000),
        ImageProcConfig(56, "square", IMAGENET_STANDARD_MEAN, IMAGENET_STANDARD_STD), image_token_id=998,
        prompt_ids=(300, 301, 302, 303), query_prefix_ids=(400, 401)),
}


def get_spec(name: str):
    if name in REGISTRY:
        return REGISTRY[name]
    if name in TINY:
        return TINY[name]
    if name in COLPALI:
        return COLPALI[name]
    raise KeyError(f"unknown model {name!r}; known: {sorted(REGISTRY) + sorted(TINY) + sorted(COLPALI)}")


def image_flops(spec: ModelSpec) -> float:
    """Algorithmic FLOPs of one image through the vision tower (GEMMs + attention, 2*M*N*K)."""
    v = spec.vision
    P = v.num_patches
    T = P + (1 if spec.family == "clip" else 0)
    d, I = v.hidden, v.intermediate
    f = 2.0 * P * (3 * v.patch * v.patch) * d
    f += v.layers * (2.0 * T * d * (3 * d + d + 2 * I) + 4.0 * T * T * d)
    if spec.family == "siglip":  # MAP head: kv proj over T tokens + tiny per-image tail
        f += 2.0 * T * d * 2 * d + 4.0 * T * d + 2.0 * d * (d + 2 * I)
    else:
        f += 2.0 * d * spec.proj_dim
    return f


def text_flops(spec: ModelSpec, L: int) -> float:
    t = spec.text
    d, I = t.hidden, t.intermediate
    f = t.layers * (2.0 * L * d * (3 * d + d + 2 * I) + 4.0 * L * L * d)
    f += 2.0 * d * spec.proj_dim
    return f


def exec_batches(spec: "ModelSpec"):
    """(image, caption) execution-batch caps of a dual-encoder job (see EXEC_IMG_BATCH above)."""
    return EXEC_IMG_BATCH, EXEC_TXT_BATCH_SIGLIP if spec.family == "siglip" else EXEC_TXT_BATCH
