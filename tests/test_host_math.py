"""Host-side (CPU) checks of the device arithmetic: compiles
tests/host/test_codelets.cpp -- which includes the kernels' own headers
(gf65537.h, fnt_codelets.h, matrix_pack.h) -- with g++ under UBSan
(signed overflow traps) and runs it.  See that file for what is checked."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_codelets_and_dot2_on_host(tmp_path):
    exe = str(tmp_path / "test_codelets")
    subprocess.check_call([
        "g++", "-std=c++20", "-O1", "-fsanitize=signed-integer-overflow,shift",
        "-fno-sanitize-recover=all", "-DQI_HOST_CHECK",
        os.path.join(HERE, "host", "test_codelets.cpp"), "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ALL OK" in r.stdout, r.stdout[-2000:]
