#!/usr/bin/env python3
"""Coefficients of the exact-erf GELU of csrc/common.h (gelu_erf2, round 6).

gelu(x) = x Phi(x) with Phi(x) = sigmoid(y(x)), y = logit(Phi) = log Phi(x) - log Phi(-x), an odd function:
y(x) ~= x P(x^2), P of degree 6 in x^2, fitted by linear programming to minimise max |dPhi| =
Phi (1 - Phi) |dy| on x in (0, 6.2] (dPhi is what the output sees; Phi(-x) = 1 - Phi(x) by oddness, so
the negative half has the same error). The device evaluates 2^(-log2(e) x P(x^2)) with v_exp_f32 and the
sigmoid with v_rcp_f32 -- the cost of the gelu_tanh form plus five fused multiply-adds, and no branch:
x P(x^2) is monotone, so |x| > 6.2 needs no clamp (v_exp_f32 saturates to 0 / +inf, v_rcp_f32(inf) = 0).

    python tools/gelu_erf_fit.py      # prints the float32 coefficients (-log2(e) folded in) and the error
"""
import numpy as np
from scipy.optimize import linprog
from scipy.special import log_ndtr, ndtr

DEG = 6
XMAX = 6.2
LOG2E = 1.4426950408889634


def fit(deg: int = DEG, xmax: float = XMAX, n: int = 9000):
    x = np.linspace(1e-5, xmax, n)
    phi = ndtr(x)
    y = log_ndtr(x) - log_ndtr(-x)
    w = phi * (1 - phi)
    A = np.stack([x ** (2 * i + 1) for i in range(deg + 1)], 1)
    m = deg + 1
    a_ub = np.vstack([np.hstack([w[:, None] * A, -np.ones((n, 1))]), np.hstack([-w[:, None] * A, -np.ones((n, 1))])])
    b_ub = np.concatenate([w * y, -w * y])
    c = np.zeros(m + 1)
    c[-1] = 1
    r = linprog(c, A_ub=a_ub, b_ub=b_ub, bounds=[(None, None)] * (m + 1), method="highs")
    return r.x[:m], r.x[-1]


def gelu_f32(x: np.ndarray, cf: np.ndarray) -> np.ndarray:
    """The device arithmetic in float32 (fused multiply-adds rounded once; exp2 / rcp correctly rounded)."""
    f = np.float32
    x = x.astype(f)
    x2 = (x * x).astype(f)
    p = np.full_like(x2, cf[-1])
    for c in cf[-2::-1]:
        p = (p.astype(np.float64) * x2 + c).astype(f)
    u = (x * p).astype(f)
    with np.errstate(over="ignore"):
        e = np.exp2(u.astype(np.float64)).astype(f)
        d = (e + f(1)).astype(f)
        r = (1.0 / d.astype(np.float64)).astype(f)
    return (x * r).astype(f)


if __name__ == "__main__":
    co, dphi = fit()
    cf = (-co * LOG2E).astype(np.float32)
    x = np.linspace(-12, 12, 2_400_001).astype(np.float32)
    ref = x.astype(np.float64) * ndtr(x.astype(np.float64))
    g = gelu_f32(x, cf)
    m = np.abs(x) > 1e-3
    erf_eq = 2 * np.abs(g - ref)[m] / np.abs(x[m])
    print(f"fit: max |dPhi| {dphi:.3g}; float32 evaluation: erf-equivalent abs error max {erf_eq.max():.3g}")
    print("coefficients (c0 .. c6 of -log2(e) x P(x^2)):")
    print(", ".join(f"{v:.9g}f" for v in cf))
