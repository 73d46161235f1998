"""The sphere test's division (render.hip div_rn: two residual corrections from RN(1/a), Markstein) is
bit-identical to IEEE x / a wherever the kernel uses it: tools/check_fastdiv.c, compiled here with gcc,
compares 2e7 random and near-tie cases (1e10 were run when the kernel adopted it)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_div_rn_matches_ieee_division(tmp_path):
    exe = str(tmp_path / "check_fastdiv")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fopenmp", os.path.join(ROOT, "tools", "check_fastdiv.c"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe, "2e7"], check=False, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout
