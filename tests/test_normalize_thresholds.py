"""k_normalize4's decisions on the squared norm (ur3e_amd/csrc/ur3e_engine.h) equal the oracle's
decisions on the norm (mju_normalize4): the constants match tools/normalize_thresholds.py and the two
tests agree on every double within 1e5 ulps of each boundary and on random squared norms."""
import math
import os
import random
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import normalize_thresholds as nt  # noqa: E402


def test_constants_match_the_kernel_source():
    src = open(os.path.join(ROOT, "ur3e_amd", "csrc", "ur3e_engine.h")).read()
    for k, v in nt.thresholds().items():
        m = re.search(r"#define %s (\S+)" % k, src)
        assert m, k
        assert float.fromhex(m.group(1)) == v, k


def test_decisions_agree():
    t = nt.thresholds()
    for base in list(t.values()) + [1.0]:
        for d in (-1, 1):
            x = base
            for _ in range(100000):
                assert nt.rescales_by_norm(x) == nt.rescales_by_square(x, t), x.hex()
                x = math.nextafter(x, math.inf if d > 0 else -math.inf)
    rng = random.Random(0)
    for _ in range(200000):
        x = rng.uniform(0, 4) * 10.0 ** rng.randint(-40, 3)
        assert nt.rescales_by_norm(x) == nt.rescales_by_square(x, t)
    for x in (0.0, math.inf):
        assert nt.rescales_by_norm(x) == nt.rescales_by_square(x, t)
    assert not nt.rescales_by_square(math.nan, t) and not nt.rescales_by_norm(math.nan)
