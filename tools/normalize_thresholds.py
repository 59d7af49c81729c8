"""Squared-norm thresholds of k_normalize4 in tools/var/nrm4sq.patch (against ur3e_amd/csrc/ur3e_engine.h).

MuJoCo's mju_normalize4 (restated by the oracle) takes n = sqrt(s), s = |q|^2, leaves q as it is when
|n - 1| <= mjMINVAL and sets it to the identity when n < mjMINVAL.  sqrt is correctly rounded and
monotonic, so both tests are equivalent to comparisons on s itself, which the kernel makes before it
takes any square root (the root is taken only in the rare rescale branch).  This script derives the
exact double thresholds; tests/test_normalize_thresholds.py checks the patch's constants
against it and brute-forces the equivalence around every boundary."""
import math

MINVAL = 1e-15


def _next(x, d):
    return math.nextafter(x, math.inf if d > 0 else -math.inf)


def thresholds():
    nlo = 1.0
    while abs(_next(nlo, -1) - 1.0) <= MINVAL:
        nlo = _next(nlo, -1)
    nhi = 1.0
    while abs(_next(nhi, 1) - 1.0) <= MINVAL:
        nhi = _next(nhi, 1)
    s = nlo * nlo
    while math.sqrt(s) >= nlo:
        s = _next(s, -1)
    while math.sqrt(s) < nlo:
        s = _next(s, 1)
    slo = s
    s = nhi * nhi
    while math.sqrt(s) <= nhi:
        s = _next(s, 1)
    while math.sqrt(s) > nhi:
        s = _next(s, -1)
    shi = s
    s = MINVAL * MINVAL
    while math.sqrt(s) >= MINVAL:
        s = _next(s, -1)
    while math.sqrt(s) < MINVAL:
        s = _next(s, 1)
    return {"K_NRM_TINY": s, "K_NRM_LO": slo, "K_NRM_HI": shi}


def rescales_by_norm(s):
    """the oracle's decision on n = sqrt(s)"""
    n = math.sqrt(s)
    return not (n < MINVAL) and abs(n - 1.0) > MINVAL


def rescales_by_square(s, t):
    """the kernel's decision on s"""
    return s >= t["K_NRM_TINY"] and (s < t["K_NRM_LO"] or s > t["K_NRM_HI"])


if __name__ == "__main__":
    for k, v in thresholds().items():
        print(k, v.hex(), repr(v))
