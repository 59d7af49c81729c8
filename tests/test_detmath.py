"""Deterministic FP64 math (ur3e_amd/csrc/detmath.h, shared by kernels and oracle)
vs glibc libm: <= 2 ulp on the ranges the hot path uses."""
import ctypes
import math

import numpy as np

from oracle import pyoracle as po


def _ulps(a, b):
    if a == b:
        return 0.0
    return abs(a - b) / (np.spacing(abs(b)) or 5e-324)


def test_detmath_accuracy():
    L = po.lib()
    L.ur3o_detmath.restype = ctypes.c_double
    f = lambda fn, x, y=0.0: L.ur3o_detmath(ctypes.c_int(fn), ctypes.c_double(x), ctypes.c_double(y))
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-40, 40, 20000), rng.uniform(-1e-3, 1e-3, 2000), [0.0, 1e-300, math.pi / 4]])
    worst = dict(sin=0, cos=0, exp=0, atan=0, atan2=0, tanh=0)
    for x in xs:
        worst["sin"] = max(worst["sin"], _ulps(f(0, x), math.sin(x)))
        worst["cos"] = max(worst["cos"], _ulps(f(1, x), math.cos(x)))
        worst["exp"] = max(worst["exp"], _ulps(f(2, x * 10), math.exp(x * 10)))
        worst["atan"] = max(worst["atan"], _ulps(f(4, x), math.atan(x)))
        y = x * 0.3 - 1
        worst["atan2"] = max(worst["atan2"], _ulps(f(5, y, x), math.atan2(y, x)))
        if abs(x) > 0.5:
            worst["tanh"] = max(worst["tanh"], _ulps(f(3, x / 8), math.tanh(x / 8)))
    for k in ("sin", "cos", "exp", "atan", "atan2"):
        assert worst[k] <= 2, (k, worst[k])
    assert worst["tanh"] <= 64, worst  # tanh via exp: ~1e-14 relative, used only in the reward
