"""The flop-counting build of the oracle (oracle/flops, bench.py's FP64 roofline) computes exactly
what the plain oracle computes (count_flops asserts equal observations every step), and counts a
plausible number of FP64 operations per env-step."""
import json
import os
import sys


def test_counting_build_matches_oracle(tmp_path):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import count_flops
    out = str(tmp_path / "flops.json")
    count_flops.main(8, 6, out_path=out)
    d = json.load(open(out))
    # 2 substeps of kinematics, collision, a Newton solve over ~13-40 rows: 1e4..1e6 FP64 ops
    assert 1e4 < d["flops_per_env_step"] < 1e6
