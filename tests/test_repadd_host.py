"""dr::rep_add (deeprec-1_amd/csrc/dr_repadd.h), the closed-form k-fold
fp32 addition the segment walker of long gradient runs uses, is bit-equal to
the plain loop of k in-order adds (the reference's serial sum,
segment_reduction_ops.cc:391-404) -- checked on the host (g++, SSE fp32,
round-to-nearest-even, no contraction) over random cases that cover ties,
binade edges, sign changes, zeros, subnormals and non-finite values
(tools/repadd_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not shutil.which("g++"), reason="g++ absent")
@pytest.mark.parametrize("seed", [1, 7, 2021])
def test_rep_add_matches_plain_loop(tmp_path, seed):
    exe = str(tmp_path / "repadd_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17",
                    "-I", os.path.join(ROOT, "deeprec-1_amd", "csrc"),
                    os.path.join(ROOT, "tools", "repadd_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "400000", str(seed)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "mismatches 0" in r.stdout
