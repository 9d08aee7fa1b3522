"""Planted retrieval embeddings, regenerable bit-for-bit on any box.

img_i = norm(base_i + noise·N), cap_{5i+j} = norm(base_i + noise·N), bf16.
numpy's PCG64 + ziggurat normals (platform independent for one numpy version),
norms in float64, one float32 rounding, then torch's round-to-nearest-even bf16
cast. The fixture that pins the reference's ranking of these embeddings
(full_retrieval.npz) also stores a checksum of the bf16 bits, so a test that
regenerates them on the GPU box proves it ranks the very same inputs.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch


def _unit_bf16(x: np.ndarray) -> torch.Tensor:
    nrm = np.sqrt((x.astype(np.float64) ** 2).sum(1, keepdims=True))
    return torch.from_numpy((x / nrm).astype(np.float32)).to(torch.bfloat16)


def planted_np(n: int, caps: int, D: int, noise: float, seed: int = 0):
    """(img [n, D] bf16, all_txt [caps·n, D] bf16); T2I captions are all_txt[::caps]."""
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n, D), dtype=np.float32)
    img = base + np.float32(noise) * rng.standard_normal((n, D), dtype=np.float32)
    cap = np.repeat(base, caps, 0) + np.float32(noise) * rng.standard_normal((n * caps, D), dtype=np.float32)
    return _unit_bf16(img), _unit_bf16(cap)


def planted_ties(n: int, caps: int, D: int, noise: float, seed: int = 0):
    """planted_np with EXACT duplicates, so exact fp32 score ties decide top-k places.

    Disjoint groups of 2, 3 or 4 images share one base (each member's captions describe the
    others too, so the tied columns rank high). Per group, by mode (cycled):
      0 'img'  every member's image is the lead's image (T2I rows tie member images);
      1 'cap0' every member's caption 0 is the lead's caption 0 (Sym rows tie T2I captions,
               I2T rows tie captions 5m);
      2 'capj' caption j = 1 + (group % 4) duplicated (I2T only);
      3 'both' images and caption 0.
    About 35 % of the images belong to a group. Returns (img [n, D] bf16, all_txt [caps·n, D]
    bf16, groups int32 [n_groups, 6] = (mode, size, lead, member, member, member; -1 padded))."""
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n, D), dtype=np.float32)
    perm = rng.permutation(n)
    groups, pos = [], 0
    for size, count in ((2, int(0.10 * n)), (3, int(0.03 * n)), (4, int(0.015 * n))):
        for _ in range(count):
            if pos + size > n:
                break
            groups.append(perm[pos:pos + size].copy())
            pos += size
    for m in groups:
        base[m] = base[m[0]]
    img = base + np.float32(noise) * rng.standard_normal((n, D), dtype=np.float32)
    cap = np.repeat(base, caps, 0) + np.float32(noise) * rng.standard_normal((n * caps, D), dtype=np.float32)
    table = np.full((len(groups), 6), -1, np.int32)
    for g, m in enumerate(groups):
        mode = g % 4
        lead = m[0]
        if mode in (0, 3):
            img[m] = img[lead]
        if mode in (1, 3):
            cap[caps * m] = cap[caps * lead]
        if mode == 2:
            j = 1 + (g // 4) % (caps - 1)
            cap[caps * m + j] = cap[caps * lead + j]
        table[g, 0], table[g, 1] = mode, len(m)
        table[g, 2:2 + len(m)] = m
    return _unit_bf16(img), _unit_bf16(cap), table


def planted_multivec(n: int, caps: int, Ld: int, qlens: tuple, noise: float, batch: int = 4, seed: int = 0):
    """ColPali-shaped planted multi-vectors (SURVEY §8d config 4 geometry, scaled down in n).

    Image i: Ld unit tokens norm(base_i + noise·N) (every row valid, as for ColPali image
    sequences). Caption c of image c // caps: len_c ∈ [qlens) unit tokens norm(base + noise·N).
    As the reference's process_queries left-pads each batch of `batch` captions to its longest
    query and the encoder zeroes padded rows (TF:models/colpali/modeling_colpali.py:139-140),
    caption c's per-item tensor has pad_c - len_c leading zero rows (pad_c = its batch's longest).
    Returns (img [n, Ld, 128] bf16, cap_valid [n·caps, max_len, 128] bf16 valid rows first,
    cap_len [n·caps] int32, cap_pad [n·caps] int32)."""
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n, 128), dtype=np.float32)
    img = base[:, None, :] + np.float32(noise) * rng.standard_normal((n, Ld, 128), dtype=np.float32)
    m = n * caps
    lens = rng.integers(qlens[0], qlens[1], m).astype(np.int32)
    Lq = int(lens.max())
    cap = np.zeros((m, Lq, 128), np.float32)
    for c in range(m):
        cap[c, : lens[c]] = base[c // caps] + np.float32(noise) * rng.standard_normal((int(lens[c]), 128),
                                                                                      dtype=np.float32)
    pad = np.array([int(lens[s:s + batch].max()) for s in range(0, m, batch) for _ in range(min(batch, m - s))],
                   np.int32)

    def unit(x):
        nrm = np.sqrt((x.astype(np.float64) ** 2).sum(-1, keepdims=True))
        return torch.from_numpy(np.where(nrm > 0, x / np.maximum(nrm, 1e-300), 0.0).astype(np.float32)).to(
            torch.bfloat16)
    return unit(img), unit(cap), torch.from_numpy(lens), torch.from_numpy(pad)


def left_padded_items(cap: torch.Tensor, lens: torch.Tensor, pad: torch.Tensor):
    """Per-item caption tensors as the reference's encode_data hands them to scoring: [pad_c, 128]
    with the pad_c - len_c leading rows zero (left padding, masked to zero by the encoder)."""
    out = []
    for c in range(cap.shape[0]):
        e = torch.zeros(int(pad[c]), cap.shape[2], dtype=cap.dtype)
        e[int(pad[c]) - int(lens[c]):] = cap[c, : int(lens[c])]
        out.append(e)
    return out


def config0_inputs(spec, n_img: int = 64, caps: int = 5, seed: int = 21):
    """BASELINE configs[0] inputs: n_img synthetic 224² u8 images and caps·n_img CLIP caption id rows
    ([bos] + 3..75 ids + [eos], ragged, so every batch of 32 pads differently)."""
    from mme.processor import synthetic_images
    t = spec.text
    imgs = synthetic_images(n_img, seed=seed)
    rng = np.random.default_rng(seed + 1)
    lens = rng.integers(3, t.max_pos - 1, caps * n_img)
    cap_rows = [[t.bos_id] + rng.integers(1, min(t.bos_id, t.eos_id), int(L)).tolist() + [t.eos_id] for L in lens]
    return imgs, cap_rows


E2E_MODELS = (("tiny-clip", 32, 112), ("tiny-siglip", 64, 112), ("OpenAI-CLIP-L", 64, 224), ("SigLIP-400M", 64, 224))
# the ViT-H towers of BASELINE configs[2] (LAION-CLIP-H), configs[3] / [4] (Apple-DFN5B-H, bf16 and fp8) and
# SURVEY §8 f4 (MetaCLIP-H14):
# their own fixture file (e2e_fitted_h.npz), so e2e_fitted.npz stays as generated
E2E_H_MODELS = (("LAION-CLIP-H", 64, 224), ("Apple-DFN5B-H", 64, 224), ("MetaCLIP-H14", 64, 224))


def e2e_inputs(spec, n: int, H: int, caps: int = 5, seed: int = 41):
    """Inputs of the end-to-end fixture (e2e_fitted.npz): n synthetic H x H u8 images and caps*n ragged
    caption id rows (CLIP: [bos] + 1..L-2 ids + [eos]; SigLIP: 1..L-1 ids + [eos]) in main.py's layout
    (caption j of image i at caps*i + j, T2I = caption 0)."""
    from mme.processor import synthetic_images
    t = spec.text
    imgs = synthetic_images(n, H, H, seed=seed)
    rng = np.random.default_rng(seed + 1)
    if t.bos_id is not None:
        lens = rng.integers(1, t.max_pos - 1, caps * n)
        rows = [[t.bos_id] + rng.integers(1, min(t.bos_id, t.eos_id), int(L)).tolist() + [t.eos_id] for L in lens]
    else:
        lens = rng.integers(1, t.max_pos, caps * n)
        rows = [rng.integers(2, t.vocab, int(L)).tolist() + [t.eos_id] for L in lens]
    return imgs, rows


GRADED_OWN_RANK = (0, 7)   # 0-based rank of the own image per caption table (t = l mod 2): R@1 50, R@5 50, R@10 100


def graded_targets(n: int, caps: int, D: int, seed: int = 0, K: int = 12, delta: float = 0.038):
    """Target joint embeddings with a GRADED score structure (the fitted projection heads of the
    end-to-end fixture map the towers' pooled features onto these; make_goldens.make_e2e).

    Image i -> u_i (orthonormal); caption (l, 0) -> sum_k L[lev_l(k)] u_{(l+k) mod n} + r u_null, so
    a T2I row, a Sym row and the top of an I2T row see the K distinct levels L = delta*(K..1), spaced
    delta apart, and every other score is 0. Caption tables t = l mod G (G = len(GRADED_OWN_RANK))
    place the own image at GRADED_OWN_RANK[t]; the level map lev_t(k) = sigma((k + G*d_t) mod K) keeps
    every Sym / I2T row a bijection onto the levels (the G residues never collide). Captions j >= 1
    carry only 0.2*j*delta of their own image (below the I2T top-11) plus u_null. Returns float64
    (img [n, D], cap [caps*n, D]) of unit norm."""
    G = len(GRADED_OWN_RANK)
    assert K % G == 0 and G * G <= K and n % G == 0 and n >= K and D >= n + 1
    rng = np.random.default_rng(seed)
    u = np.linalg.qr(rng.standard_normal((D, n + 1)))[0].T        # [n+1, D] orthonormal; u[n] = u_null
    L = delta * np.arange(K, 0, -1, dtype=np.float64)             # level value by rank 0..K-1
    assert (L ** 2).sum() < 1.0
    # sigma: a fixed bijection of level indices with sigma(G*d_t) = own rank of table t
    d = list(range(G))
    sigma = {G * dt: GRADED_OWN_RANK[t] for t, dt in enumerate(d)}
    rest_src = [x for x in range(K) if x not in sigma]
    rest_dst = [x for x in range(K) if x not in sigma.values()]
    perm = rng.permutation(len(rest_dst))
    sigma.update({s: rest_dst[p] for s, p in zip(rest_src, perm)})
    img = u[:n].copy()
    cap = np.zeros((caps * n, D))
    for l in range(n):
        t = l % G
        lev = [sigma[(k + G * d[t]) % K] for k in range(K)]
        v = np.array([L[x] for x in lev])
        cap[caps * l] = v @ u[(l + np.arange(K)) % n] + np.sqrt(1.0 - (v ** 2).sum()) * u[n]
        for j in range(1, caps):
            a = 0.2 * j * delta
            cap[caps * l + j] = a * u[l] + np.sqrt(1.0 - a * a) * u[n]
    return img, cap


def bf16_sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().view(torch.int16).numpy().tobytes()).hexdigest()[:32]
