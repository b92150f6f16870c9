#!/usr/bin/env python3
"""Polynomial coefficients of csrc/detmath_fast.h (near-minimax Chebyshev
fits by mpmath.chebyfit at 120 bits, rounded to double), with the fit's max
relative error.  Session tool: the header holds the printed constants."""
import mpmath as mp

mp.mp.prec = 120


def fit(name, f, a, b, deg, rel=None):
    coeffs, err = mp.chebyfit(f, [a, b], deg + 1, error=True)
    # relative max error over a dense grid, after rounding coefficients to double
    cd = [float(c) for c in coeffs]        # highest degree first
    worst = mp.mpf(0)
    for i in range(2001):
        x = a + (b - a) * mp.mpf(i) / 2000
        p = mp.mpf(0)
        for c in cd:
            p = p * x + mp.mpf(c)
        ref = f(x)
        den = abs(rel(x)) if rel else abs(ref)
        if den != 0:
            worst = max(worst, abs(p - ref) / den)
    print(f"/* {name}: degree {deg} on [{float(a):.6g}, {float(b):.6g}], max rel err 2^{float(mp.log(worst, 2)):.1f} */")
    print("  " + ", ".join(c.hex() for c in cd))
    return cd


L2 = mp.log(2)
# exp(r), |r| <= ln2/2
for d in (8, 9):
    fit(f"exp deg{d}", mp.exp, -L2 / 2 - mp.mpf(1e-6), L2 / 2 + mp.mpf(1e-6), d)
# atan(t)/t in z = t^2, |t| <= tan(pi/8)
zt = mp.tan(mp.pi / 8) ** 2 * (1 + mp.mpf(1e-9))
def atan_q(z):
    if z == 0:
        return mp.mpf(1)
    t = mp.sqrt(z)
    return mp.atan(t) / t
for d in (8, 9, 10):
    fit(f"atan deg{d}", atan_q, mp.mpf(0), zt, d)
# sin(r)/r and cos(r) in z = r^2, |r| <= pi/4 (+ margin)
zr = (mp.pi / 4 * (1 + mp.mpf(1e-6))) ** 2
def sin_q(z):
    if z == 0:
        return mp.mpf(1)
    r = mp.sqrt(z)
    return mp.sin(r) / r
def cos_q(z):
    return mp.cos(mp.sqrt(z))
for d in (5, 6):
    fit(f"sin/r deg{d}", sin_q, mp.mpf(0), zr, d)
    fit(f"cos deg{d}", cos_q, mp.mpf(0), zr, d)
# log(m) = 2 s P(s^2), s = (m - 1) / (m + 1), |s| <= (sqrt2 - 1) / (sqrt2 + 1)
zs = ((mp.sqrt(2) - 1) / (mp.sqrt(2) + 1)) ** 2 * (1 + mp.mpf(1e-6))
def atanh_q(z):
    if z == 0:
        return mp.mpf(1)
    s = mp.sqrt(z)
    return mp.atanh(s) / s
for d in (5, 6, 7):
    fit(f"atanh deg{d}", atanh_q, mp.mpf(0), zs, d)
# sinh(a) = a + a z S(z), |a| < 1: fit sinh(a)/a in z
def sinh_q(z):
    if z == 0:
        return mp.mpf(1)
    a = mp.sqrt(z)
    return mp.sinh(a) / a
for d in (6, 7, 8):
    fit(f"sinh/a deg{d}", sinh_q, mp.mpf(0), mp.mpf(1), d)

# Round 6: the ambiguous band is 2^13 units of the double's last place (error
# budget 2^-40 relative, detmath_fast.h), so lower degrees suffice.
print("/* ---- round 6 fits (budget 2^-40) ---- */")
# (exp(r) - 1) / r, |r| <= ln2/512 (the 256-entry table of 2^(j/256))
def expm1_q(r):
    if r == 0:
        return mp.mpf(1)
    return mp.expm1(r) / r
rr = L2 / 512 * (1 + mp.mpf(1e-6))
for d in (2, 3):
    fit(f"expm1/r deg{d} (table 256)", expm1_q, -rr, rr, d, rel=lambda r: mp.exp(r) / (abs(r) if r != 0 else 1) if r != 0 else 1)
for d in (6, 7):
    fit(f"atan deg{d}", atan_q, mp.mpf(0), zt, d)
for d in (4, 5):
    fit(f"sin/r deg{d}", sin_q, mp.mpf(0), zr, d)
    fit(f"cos deg{d}", cos_q, mp.mpf(0), zr, d)
for d in (4,):
    fit(f"atanh deg{d}", atanh_q, mp.mpf(0), zs, d)
for d in (5,):
    fit(f"sinh/a deg{d}", sinh_q, mp.mpf(0), mp.mpf(1), d)
