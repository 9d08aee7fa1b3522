import numpy as np
import torch


def bits_to_bf16(bits: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(bits).view(np.int16)).view(torch.bfloat16)


def bits_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.detach().to("cpu", torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


def row_cos(a, b):
    a = torch.as_tensor(a).float()
    b = torch.as_tensor(b).float()
    return torch.nn.functional.cosine_similarity(a, b, dim=-1)
