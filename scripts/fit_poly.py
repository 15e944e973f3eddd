"""Fit the f64 polynomials of the two-class fast path (csrc/optimize_kernels.h).

    python scripts/fit_poly.py

exp(r) on [-ln2/2, ln2/2], degree 10 (c0 forced to 1 so exp(0) == 1), and
g(u) = atanh(sqrt u)/sqrt u on [0, (3 - 2 sqrt 2)^2] (s = (m-1)/(m+1) with
m in [1, sqrt 2)), degree 6.  Least squares at Chebyshev nodes
(near-minimax); prints the coefficients and max relative errors.
"""
import math

import numpy as np
from numpy.polynomial import chebyshev as C
from numpy.polynomial import polynomial as P


def fit_monomial(f, a, b, deg, n=4000):
    k = np.arange(n)
    x = np.cos((2 * k + 1) / (2 * n) * np.pi)
    t = (x + 1) / 2 * (b - a) + a
    c = C.chebfit(x, np.array([f(v) for v in t]), deg)
    p = C.cheb2poly(c)
    s, o = 2 / (b - a), -(a + b) / (b - a)
    mon = np.zeros(deg + 1)
    for kk, pk in enumerate(p):
        term = P.polypow([o, s], kk)
        mon[:len(term)] += pk * term
    return mon


def horner(c, x):
    q = c[-1]
    for k in range(len(c) - 2, -1, -1):
        q = q * x + c[k]
    return q


def main():
    h = math.log(2) / 2
    exp_c = fit_monomial(math.exp, -h, h, 10)
    exp_c[0] = 1.0
    r = np.linspace(-h, h, 200001)
    print('exp  deg10 max rel err %.2e' % np.max(np.abs(horner(exp_c, r) / np.exp(r) - 1)))
    print('kExpCoef =', ', '.join(repr(float(v)) for v in exp_c))
    umax = (3 - 2 * math.sqrt(2)) ** 2

    def g(u):
        return 1.0 if u == 0 else math.atanh(math.sqrt(u)) / math.sqrt(u)

    log_c = fit_monomial(g, 0.0, umax, 6)
    us = np.linspace(0, umax, 100001)
    ref = np.array([g(u) for u in us])
    print('atanh deg6 max rel err %.2e' % np.max(np.abs(horner(log_c, us) / ref - 1)))
    print('kLogCoef =', ', '.join(repr(float(v)) for v in log_c))


if __name__ == '__main__':
    main()
