"""The step kernels divide by a body's m and k and by a contact's |u_t|
through their reciprocals (rb_device.hpp div_by / div3_by: Markstein's
correction step, IEEE division outside the safe exponent range).  That is
bit-exact only if the correction step always yields RN(a / b): checked here
on the host (the same operations, with fma) against the division on random
pairs of both precisions; the GPU suite checks the kernels against the
oracle and the reference's KATs."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_reciprocal_division_is_the_ieee_division(tmp_path):
    exe = tmp_path / "div_check"
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "scripts", "div_check.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout, r.stdout
