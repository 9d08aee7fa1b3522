"""mme — MI355X-native multimodal-embedding retrieval engine (gfx950).

Hot path of sariekr/multimodal-embedding main.py (encode -> L2-normalise ->
similarity -> top-k recall, plus ColPali MaxSim) on hand-written HIP kernels
in libmme.so (include/mme.h), driven from Python over PyTorch-ROCm memory.
"""
from .config import REGISTRY, TINY, ModelSpec, get_spec  # noqa: F401
from .models import CLIPModel, SiglipModel, load_model  # noqa: F401

__version__ = "0.1.0"
