"""k_div_rcp (ur3e_amd/csrc/ur3e_engine.h), the Newton triangular sweeps' division by the Cholesky
pivot from its reciprocal, is the correctly rounded quotient: tools/div_rcp_check.c compares it with
n / d bit for bit on the host (the GPU sweeps are compared with the oracle by the -m gpu parity tests)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_div_rcp_bit_exact(tmp_path):
    exe = str(tmp_path / "drc")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tools", "div_rcp_check.c"),
                    "-lm", "-o", exe], check=True)
    out = subprocess.run([exe, "20000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert "bad=0" in out.stdout
