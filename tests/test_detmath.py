"""Accuracy of the shared deterministic transcendentals (include/as_detmath.h).

The HIP kernels and the CPU oracle evaluate atan2 / asin / exp / sin / cos through these functions
(built from correctly rounded +, *, fmaf, division and sqrtf only), which is what makes observations
and rewards bit-identical between them (tests/test_gpu_exact.py).  Here, on the host, their error
against float64 numpy is bounded in ulps of the float32 result, over the domains the task uses, and
the signed-zero / boundary cases follow C's atan2 and torch.remainder.
"""

import ctypes as C

import numpy as np


def _eval(orc, fn, a, b=None):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(a if b is None else b, np.float32)
    out = np.zeros_like(a)
    fp = C.POINTER(C.c_float)
    orc.L.or_detmath_eval(C.c_int(fn), C.c_int(len(a)), a.ctypes.data_as(fp), b.ctypes.data_as(fp),
                          out.ctypes.data_as(fp))
    return out


def _ulps(got, ref):
    ref32 = ref.astype(np.float32)
    ulp = np.spacing(np.abs(ref32)).astype(np.float64)
    ulp = np.maximum(ulp, np.float64(np.spacing(np.float32(1e-30))))
    return np.abs(got.astype(np.float64) - ref) / ulp


def test_atan2_accuracy(orc):
    rng = np.random.default_rng(0)
    ang = rng.uniform(-np.pi, np.pi, 200_000)
    r = np.exp(rng.uniform(-6, 3, ang.size))
    y = (r * np.sin(ang)).astype(np.float32)
    x = (r * np.cos(ang)).astype(np.float32)
    got = _eval(orc, 0, y, x)
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert _ulps(got, ref).max() <= 3.0, _ulps(got, ref).max()


def test_atan2_special_cases(orc):
    y = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0, 1.0, -1.0, 1e-30, 5.0], np.float32)
    x = np.array([0.0, 0.0, -0.0, -0.0, 0.0, 0.0, -0.0, -0.0, -1.0, 5.0], np.float32)
    got = _eval(orc, 0, y, x)
    ref = np.arctan2(y, x).astype(np.float32)
    assert np.array_equal(np.signbit(got), np.signbit(ref))
    np.testing.assert_allclose(got, ref, rtol=3e-7, atol=0)


def test_asin_accuracy(orc):
    s = np.concatenate([np.random.default_rng(1).uniform(-1, 1, 200_000), [0.5, -0.5, 0.4999999, 0.9999999]])
    s = s.astype(np.float32)
    s = s[np.abs(s) < 1]
    got = _eval(orc, 1, s)
    ref = np.arcsin(s.astype(np.float64))
    assert _ulps(got, ref).max() <= 3.0, _ulps(got, ref).max()
    assert np.signbit(_eval(orc, 1, np.array([-0.0], np.float32)))[0]


def test_exp_accuracy(orc):
    x = np.random.default_rng(2).uniform(-87, 0, 200_000).astype(np.float32)
    got = _eval(orc, 2, x)
    ref = np.exp(x.astype(np.float64))
    assert _ulps(got, ref).max() <= 2.0, _ulps(got, ref).max()
    assert _eval(orc, 2, np.array([0.0], np.float32))[0] == 1.0
    assert _eval(orc, 2, np.array([-100.0], np.float32))[0] == 0.0


def test_sincos_accuracy(orc):
    x = np.random.default_rng(3).uniform(-50, 50, 200_000).astype(np.float32)
    for fn, ref in ((3, np.sin), (4, np.cos)):
        got = _eval(orc, fn, x)
        r = ref(x.astype(np.float64))
        err = np.abs(got.astype(np.float64) - r)
        assert err.max() < 4e-7, (fn, err.max())  # absolute: the results are O(1)


def test_rem2pi_matches_torch_remainder(orc):
    import torch

    a = np.concatenate([np.random.default_rng(4).uniform(-np.pi, np.pi, 10_000), [0.0, -0.0, -1e-30, np.pi]])
    a = a.astype(np.float32)
    got = _eval(orc, 5, a)
    ref = torch.remainder(torch.from_numpy(a), 2 * np.pi).numpy()
    assert np.array_equal(got, ref)
