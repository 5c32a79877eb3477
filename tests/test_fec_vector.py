"""The reference's FEC round-trip unit test (test/fec_utest.cpp:38-95,
TestFnt / TestFntSys :132-156: k = 3, m = 3, 1000 random codewords each
decoded from a random k-subset) ported onto qi::fec::RsFnt's horizontal
API (encode(Vector), init_context_dec, decode(context, Vector)) through the
device path, plus Buffers round trips checked against the block API
(tests/host/fec_vector_test.cpp, built next to the library)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "fec_vector_test")


@pytest.mark.gpu
def test_fec_vector_roundtrip():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "fec_vector_test: ok" in r.stdout
