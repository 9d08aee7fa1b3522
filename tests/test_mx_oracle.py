"""CPU checks of the MX-fp8 oracle (oracle/mx.py) — the checker the GPU fp8 tests rely on."""
import numpy as np

from oracle import mx


def test_e4m3_encode_is_nearest_even():
    tab = mx.e4m3_table()
    valid = np.array([v for v in range(256) if (v & 0x7F) != 0x7F])
    vals = tab[valid]
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(4000) * np.exp2(rng.integers(-12, 10, 4000))).astype(np.float32)
    x = np.concatenate([x, vals[np.isfinite(vals)], [448.0, -448.0, 1000.0, -1e6, 0.0]]).astype(np.float32)
    q = mx.encode_e4m3(x)
    xc = np.clip(x, -448, 448)
    for xi, qi in zip(xc, q):
        d = np.abs(vals - xi)
        best = valid[d == d.min()]
        # ties -> even mantissa; +-0 are the same value
        ok = {int(b) for b in best if (b & 1) == 0} or {int(b) for b in best}
        assert int(qi) in ok or (tab[qi] == 0 and xi == 0) or tab[qi] in {float(tab[b]) for b in ok}, (xi, qi)


def test_scale_rule_is_smallest_power_of_two():
    rng = np.random.default_rng(1)
    a = np.abs(rng.standard_normal(5000) * np.exp2(rng.integers(-20, 20, 5000))).astype(np.float32)
    a = np.concatenate([a, np.float32([448.0, 449.0, 1.0, 1.75, 1.7500001, 2.0 ** -100])])
    sb = mx.scale_bytes(a).astype(np.int64)
    assert np.all(a * np.exp2(127.0 - sb) <= 448.0)
    # one step smaller would overflow 448 (unless clamped at the smallest byte)
    smaller = a * np.exp2(127.0 - (sb - 1))
    assert np.all((smaller > 448.0) | (sb == 1))
    assert mx.scale_bytes(np.float32([0.0]))[0] == 127


def test_quantize_roundtrip_error():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((37, 256)).astype(np.float32) * np.exp2(rng.integers(-6, 6, (37, 1)))
    q, planes = mx.quantize(x)
    assert q.shape == (37, 256) and planes.shape == (8, 256)
    y = mx.dequantize(q, planes, 37)
    blk = np.abs(x.reshape(37, 8, 32)).max(axis=2)
    # e4m3 keeps 3 mantissa bits: |err| <= 2^-4 |x| for normals, plus the subnormal floor of the block
    floor = np.repeat(blk * 2.0 ** -12, 32, axis=1)
    assert np.all(np.abs(y - x) <= np.abs(x) * 2.0 ** -4 + floor)


def test_gemm_ref_matches_dequantised_product():
    rng = np.random.default_rng(3)
    a = rng.standard_normal((20, 64)).astype(np.float32)
    b = rng.standard_normal((12, 64)).astype(np.float32)
    aq, asc = mx.quantize(a)
    bq, bsc = mx.quantize(b)
    ref = mx.gemm_ref(aq, asc, 20, bq, bsc, 12)
    # e4m3 keeps ~2^-4 relative precision per element: the product error is a few % of its rms
    assert np.abs(ref - a @ b.T).max() <= 0.2 * np.sqrt(np.mean((a @ b.T) ** 2))
