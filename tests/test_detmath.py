"""The deterministic transcendentals (mitsuba-alvrl_amd/csrc/detmath.h) that
the oracle, the host tracer and the strict device kernels share.

They stand in for the float libm calls of the reference's samplers and media
(math::fastexp / fastlog, include/mitsuba/core/math.h:175-199; atanf / tanf in
KullaSampling, vrlIntegrator.cpp:889-914; asinhf / sinhf in
sampleVtoDistance, :916-957).  Pinned here against the correctly rounded float
value from mpmath (120-bit evaluation, then rounded to nearest float,
subnormals included): at most one ulp anywhere, and the correctly rounded value
for all but a few parts per million of the inputs.  The device copies are
checked bit for bit against these in tests/test_gpu_strict.py.
"""
import numpy as np
import pytest

mp = pytest.importorskip("mpmath")

N = 6000


def _cr(fn, xs):
    f = {"exp": mp.exp, "log": mp.log, "atan": mp.atan, "tan": mp.tan, "asinh": mp.asinh,
         "sinh": mp.sinh}[fn]
    out = np.empty(len(xs), np.float32)
    tiny = mp.mpf(2) ** -149
    for i, x in enumerate(xs):
        with mp.workprec(120):
            v = f(mp.mpf(float(x)))
            if mp.isinf(v) or abs(v) >= mp.mpf(2) ** 128:
                out[i] = np.float32(np.inf) * (1 if v > 0 else -1)
                continue
            if abs(v) < mp.mpf(2) ** -126:          # float subnormal: fixed quantum 2^-149
                out[i] = np.float32(float(mp.nint(v / tiny) * tiny))
                continue
        with mp.workprec(24):
            v = +v
        out[i] = np.float32(float(v))
    return out


def _domain(fn, rng, n):
    sgn = rng.choice([-1.0, 1.0], n - n // 2)
    return {
        "exp": lambda: np.concatenate([rng.uniform(-110, 95, n // 2), rng.uniform(-3, 3, n - n // 2)]),
        "log": lambda: np.concatenate([np.exp(rng.uniform(-100, 88, n // 2)), rng.uniform(0.5, 2, n - n // 2)]),
        "atan": lambda: np.concatenate([rng.uniform(-3, 3, n // 2), np.exp(rng.uniform(-30, 30, n - n // 2)) * sgn]),
        "tan": lambda: np.concatenate([rng.uniform(-1.5707963, 1.5707963, n // 2), rng.uniform(-1e-3, 1e-3, n - n // 2)]),
        "asinh": lambda: np.concatenate([rng.uniform(-4, 4, n // 2), np.exp(rng.uniform(-40, 40, n - n // 2)) * sgn]),
        "sinh": lambda: np.concatenate([rng.uniform(-1.2, 1.2, n // 2), rng.uniform(-95, 95, n - n // 2)]),
    }[fn]().astype(np.float32)


@pytest.mark.parametrize("fn", ["exp", "log", "atan", "tan", "asinh", "sinh"])
def test_detmath_correctly_rounded(oracle, fn):
    rng = np.random.default_rng(20261018 + len(fn))
    xs = _domain(fn, rng, N)
    ref = _cr(fn, xs)
    got = oracle.detmath(fn, xs)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin), fn
    assert np.array_equal(got[~fin], ref[~fin]), fn
    a = ref[fin].view(np.int32).astype(np.int64)
    b = got[fin].view(np.int32).astype(np.int64)
    ulp = np.abs(a - b)
    print(f"{fn}: {int((ulp != 0).sum())} of {fin.sum()} not correctly rounded, max {ulp.max()} ulp")
    assert ulp.max() <= 1, fn
    assert (ulp != 0).sum() <= max(1, fin.sum() // 100000), fn


def test_detmath_special_values(oracle):
    inf, nan = np.float32(np.inf), np.float32(np.nan)
    x = np.array([0.0, -0.0, inf, -inf, nan], np.float32)
    e = oracle.detmath("exp", x)
    assert e[0] == 1 and e[1] == 1 and e[2] == inf and e[3] == 0 and np.isnan(e[4])
    lg = oracle.detmath("log", np.array([0.0, -1.0, inf, 1.0], np.float32))
    assert lg[0] == -inf and np.isnan(lg[1]) and lg[2] == inf and lg[3] == 0
    at = oracle.detmath("atan", x)
    assert at[0] == 0 and at[2] == np.float32(np.pi / 2) and at[3] == -np.float32(np.pi / 2) and np.isnan(at[4])
    ash = oracle.detmath("asinh", x)
    assert ash[2] == inf and ash[3] == -inf and np.isnan(ash[4])
    sh = oracle.detmath("sinh", x)
    assert sh[2] == inf and sh[3] == -inf and np.isnan(sh[4])
    t = oracle.detmath("tan", x)
    assert t[0] == 0 and np.isnan(t[2]) and np.isnan(t[4])
