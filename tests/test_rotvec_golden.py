"""get_site_xrotvec (utils/utils.py:158-162, scipy Rotation.from_matrix(...).as_rotvec()): the oracle's
restatement against golden vectors scipy 1.15.3 produced here (tools/make_rotvec_golden.py).  The
restatement uses the project's deterministic sin/atan2 (detmath.h), scipy libm's, so the bar is 1e-12
(as for get_rot_err); the GPU matches the oracle bit for bit (tests/test_gpu_c3_record.py)."""
import os

import numpy as np

from oracle import pyoracle as po

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rotvec_from_matrix.npz")


def test_rotvec_from_matrix_matches_scipy():
    g = np.load(GOLDEN)
    assert str(g["scipy_version"]) == "1.15.3"
    for xm, rv in zip(g["xmat"], g["rotvec"]):
        np.testing.assert_allclose(po.rotvec_from_matrix(xm), rv, rtol=0, atol=1e-12)
