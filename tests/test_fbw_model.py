"""The wave-parallel fallbackQSort3 partition (fbw_partition, bz2_bwt.hip) is a
closed form of the serial partition step (bz:blocksort.c:93-180); its host
model (tools/fbw_check.cpp, the same passes as plain loops) must reproduce the
serial step's permutation and sub-ranges on 200k random ranges."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_fbw_partition_model(tmp_path):
    exe = str(tmp_path / "fbw_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "fbw_check.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout
