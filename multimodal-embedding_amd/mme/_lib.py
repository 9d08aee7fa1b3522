"""ctypes binding of libmme.so — the C ABI declared in include/mme.h.

The library is built in-tree (``make -C multimodal-embedding_amd``) so it
travels with the repository. There is deliberately NO fallback: if the
library is missing or fails to load, every compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# MME_DEV=1 loads the development build (every dev / diagnostic kernel form; `make dev`)
DEV = os.environ.get("MME_DEV", "0") == "1"
LIB_PATH = os.environ.get("MME_LIB", os.path.join(_HERE, "libmme_dev.so" if DEV else "libmme.so"))

# MME_ACT_* / MME_PIX_* from include/mme.h
ACT_NONE, ACT_GELU_TANH, ACT_QUICK_GELU, ACT_GELU_ERF, ACT_GEGLU_TANH = 0, 1, 2, 3, 4
PIX_F32_NCHW, PIX_PATCHES = 0, 1
ABI_VERSION = 9
BUILD_DEV = 1  # MME_BUILD_DEV

# name -> (restype, argtypes)
_P = c_void_p
SIGNATURES = {
    "mme_last_error": (ctypes.c_char_p, []),
    "mme_abi_version": (c_int, []),
    "mme_build_flags": (c_int, []),
    "mme_preprocess_workspace_bytes": (c_size_t, [c_int] * 5),
    "mme_preprocess_u8": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _P, _P, c_int, c_int,
                                  c_int, _P, _P, c_size_t, _P]),
    "mme_im2col": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, _P, _P]),
    "mme_gemm": (c_int, [_P, c_int, _P, c_int, _P, c_int, c_int, c_int, c_int, _P, _P, c_int, c_int, c_int, c_int,
                         _P]),
    "mme_gemm_lnfold": (c_int, [_P, c_int, _P, c_int, _P, c_int, c_int, c_int, c_int, _P, _P, _P, c_int, _P]),
    "mme_rowstats": (c_int, [_P, c_int, c_int, c_int, c_float, _P, _P]),
    "mme_gemm_res_stats": (c_int, [_P, c_int, _P, c_int, _P, c_int, c_int, c_int, c_int, _P, _P, c_int, c_float, _P,
                                   _P, _P]),
    "mme_layernorm": (c_int, [_P, c_int, _P, _P, _P, c_int, c_int, c_int, c_float, _P, _P]),
    "mme_attention": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P, c_int, c_float, _P]),
    "mme_attention_qs": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P, c_int, _P]),
    "mme_probe_attention": (c_int, [_P, _P, c_int, _P, c_int, c_int, c_int, c_int, c_int, c_float, _P]),
    "mme_map_pool": (c_int, [_P, c_int, _P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P]),
    "mme_token_embed": (c_int, [_P, c_int, c_int, _P, _P, c_int, _P, c_int, _P]),
    "mme_clip_embed_ln": (c_int, [_P, c_int, _P, _P, _P, _P, c_float, _P, c_int, c_int, c_int, c_int, _P]),
    "mme_text_pool_rows": (c_int, [_P, c_int, c_int, c_int64, c_int, _P, _P]),
    "mme_l2norm": (c_int, [_P, c_int, _P, c_int, c_int, c_int, _P]),
    "mme_sim_topk_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mme_sim_topk": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, c_int, _P, _P, _P, c_size_t, _P]),
    "mme_topk_merge": (c_int, [_P, _P, c_int, c_int, c_int, _P, _P, _P]),
    "mme_gather_scores": (c_int, [_P, ctypes.c_long, _P, _P, c_int, c_int, c_int, c_int, _P, _P]),
    "mme_recall_hits_groups": (c_int, [_P, c_int, c_int, c_int, c_int, _P, c_int, _P, _P]),
    "mme_winoground": (c_int, [_P, _P, c_int, c_int, _P, _P, _P]),
    "mme_topk_rows": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, _P, _P, _P]),
    "mme_topk_rows_torch_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mme_topk_rows_torch": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, _P, _P, _P, c_size_t, _P]),
    "mme_recall_hits": (c_int, [_P, c_int, c_int, _P, c_int, c_int, _P, c_int, _P, _P, _P]),
    "mme_tie_rows": (c_int, [_P, c_int, c_int, _P, _P]),
    "mme_sim_scores": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, _P, ctypes.c_long, _P]),
    "mme_maxsim_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "mme_maxsim": (c_int, [_P, _P, c_int, c_int, _P, _P, _P, c_int, c_int, c_int, _P, _P, c_size_t, _P]),
    "mme_mx_quant": (c_int, [_P, c_int, c_int, c_int, _P, c_int, _P, c_int, _P]),
    "mme_layernorm_mx": (c_int, [_P, c_int, _P, _P, c_int, c_int, c_float, _P, _P, c_int, _P, c_int, _P]),
    "mme_gemm_mx": (c_int, [_P, c_int, _P, c_int, _P, c_int, _P, c_int, _P, c_int, _P, c_int, c_int, c_int, c_int,
                            _P, _P, c_int, c_int, c_int, c_int, _P]),
    "mme_rmsnorm": (c_int, [_P, c_int, _P, _P, c_int, c_int, c_int, c_float, c_int, _P, _P]),
    "mme_rope": (c_int, [_P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, _P]),
    "mme_gemma_embed": (c_int, [_P, c_int, c_int, _P, c_int, c_float, _P, c_int, c_int, _P, c_int, _P]),
    "mme_l2norm_masked": (c_int, [_P, c_int, _P, c_int, c_int, c_int, _P, _P]),
    "mme_attention_mqa": (c_int, [_P, c_int, _P, c_int, c_int, c_int, c_int, c_int, _P, _P, c_float, _P]),
}
# per-call kernel forms (ABI 8; mme.ops.kernel_forms): the entry point's arguments after an int form
for _name in ("mme_gemm", "mme_gemm_lnfold", "mme_gemm_res_stats", "mme_attention", "mme_attention_qs", "mme_gemm_mx"):
    SIGNATURES[_name + "_form"] = (c_int, [c_int] + SIGNATURES[_name][1])


class MMEError(RuntimeError):
    """A libmme call returned a non-zero status."""


_lib = None


def _build() -> None:
    """Compile the in-tree library with hipcc (a checkout without the built .so)."""
    import subprocess
    pkg = os.path.dirname(_HERE)
    if os.path.exists(os.path.join(pkg, "Makefile")):
        subprocess.run(["make", "-C", pkg, "-j", str(min(16, os.cpu_count() or 8))] + (["dev"] if DEV else []),
                       check=False, stdout=subprocess.DEVNULL)


def load() -> ctypes.CDLL:
    """Load libmme.so once and bind every entry point; raise loudly on failure."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH) and os.environ.get("MME_AUTOBUILD", "1") != "0":
        _build()
    if not os.path.exists(LIB_PATH):
        raise MMEError(
            f"libmme.so not found at {LIB_PATH}; build it with `make -C multimodal-embedding_amd` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    # version first: a stale library would otherwise fail below on a missing symbol
    lib.mme_abi_version.restype, lib.mme_abi_version.argtypes = c_int, []
    if lib.mme_abi_version() != ABI_VERSION:
        raise MMEError(f"libmme ABI {lib.mme_abi_version()} at {LIB_PATH} != expected {ABI_VERSION}: stale "
                       "library, rebuild with `make -C multimodal-embedding_amd`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise MMEError(f"{LIB_PATH} does not export {name}: rebuild with `make -C multimodal-embedding_amd`")
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def is_dev() -> bool:
    """True when the loaded library is the development build (dev kernel forms compiled in)."""
    return bool(load().mme_build_flags() & BUILD_DEV)


def call(name: str, *args) -> None:
    """Invoke an int-returning entry point and raise MMEError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.mme_last_error().decode(errors="replace")
        raise MMEError(f"{name} failed (status {rc}): {msg}")


def query(name: str, *args):
    """Invoke a value-returning entry point (workspace sizes, versions)."""
    return getattr(load(), name)(*args)
