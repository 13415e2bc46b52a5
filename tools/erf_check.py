"""Accuracy of the kernels' branch-free erf (cet_device.hpp erf_rational) in fp32 arithmetic
(the reciprocal rounded to fp32, as v_rcp_f32 within 1 ulp) against the exact erf, and of the
GELU built on it:  python tools/erf_check.py"""
import math

import numpy as np

A = [-2.72614225801306e-10, 2.77068142495902e-08, -2.10102402082508e-06, -5.69250639462346e-05,
     -7.34990630326855e-04, -2.95459980854025e-03, -1.60960333262415e-02]
B = [-1.45660718464996e-05, -2.13374055278905e-04, -1.68282697438203e-03, -7.37332916720468e-03,
     -1.42647390514189e-02]


def erf_rational(x):
    f = np.float32
    xc = np.clip(x, -4, 4).astype(f)
    x2 = (xc * xc).astype(f)
    p = f(A[0])
    for c in A[1:]:
        p = (p * x2 + f(c)).astype(f)
    q = f(B[0])
    for c in B[1:]:
        q = (q * x2 + f(c)).astype(f)
    return (xc * p * (f(1) / q).astype(f)).astype(f)


if __name__ == "__main__":
    x = np.linspace(-8, 8, 400001).astype(np.float32)
    ref = np.array([math.erf(float(v)) for v in x])
    e = erf_rational(x)
    g = 0.5 * x.astype(np.float64) * (1 + np.array([math.erf(float(v) / math.sqrt(2)) for v in x]))
    gf = (np.float32(0.5) * x * (np.float32(1) + erf_rational((x * np.float32(0.70710678118654752)).astype(np.float32))))
    print(f"erf max |err| {np.abs(e - ref).max():.3g}; gelu max |err| {np.abs(gf - g).max():.3g}")
