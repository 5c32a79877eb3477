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


def _perm(src0, src1, sel):
    """v_perm_b32: result byte i = byte sel_i of the 8-byte {src0:src1}
    (selectors 0-3: src1, 4-7: src0, 0x0c: zero)."""
    b = [(src1 >> (8 * j)) & 0xff for j in range(4)] + [(src0 >> (8 * j)) & 0xff for j in range(4)]
    out = 0
    for i in range(4):
        s = (sel >> (8 * i)) & 0xff
        out |= (b[s] if s < 8 else 0) << (8 * i)
    return out


def test_split_i8_by_permutes():
    """The context kernels' byte split (ctx.hip split_i8_x4, the k <= 128 row
    pass) against matrix_pack.h's split_i8 for every canonical residue:
    b = the sign-extended low byte of v, a's byte = byte 1 of v - b, and the
    four entries' bytes gathered by three byte permutes per word; plus the
    min3 canonical form and coef_bad of the same pass."""
    import numpy as np
    q = 65537
    e = np.arange(q, dtype=np.int64)
    bal = np.where(e > 32768, e - q, e)
    v = np.where(bal > 32639, bal - q, bal)
    # split_i8 (matrix_pack.h)
    b_ref = ((v + 128) & 255) - 128
    a_ref = (v - b_ref) // 256
    # the kernel's form
    b = ((v & 0xff) ^ 0x80) - 0x80                   # (v << 24) >> 24
    va = (v - b) & 0xffffffff
    assert np.array_equal(b, b_ref)
    assert np.array_equal((va >> 8) & 0xff, a_ref & 0xff)
    assert np.array_equal(v & 0xff, b_ref & 0xff)
    # the permutes, on a few groups of four (incl. the extremes)
    rng = np.random.default_rng(5)
    groups = [np.array([0, 32640, 32767, 65536])] + [rng.integers(0, q, 4) for _ in range(200)]
    for grp in groups:
        vv = [int(v[x]) & 0xffffffff for x in grp]
        vb = vv
        vaa = [(int(v[x]) - int(b[x])) & 0xffffffff for x in grp]
        bw = _perm(_perm(vb[3], vb[2], 0x0c0c0400), _perm(vb[1], vb[0], 0x0c0c0400), 0x05040100)
        aw = _perm(_perm(vaa[3], vaa[2], 0x0c0c0501), _perm(vaa[1], vaa[0], 0x0c0c0501), 0x05040100)
        for jb, x in enumerate(grp):
            assert (bw >> (8 * jb)) & 0xff == int(b_ref[x]) & 0xff
            assert (aw >> (8 * jb)) & 0xff == int(a_ref[x]) & 0xff
    # min3 canonical form of fold(y) in [-q, 2q)
    f = np.arange(-q, 2 * q, dtype=np.int64)
    fu = f & 0xffffffff
    c = np.minimum(np.minimum(fu, (fu + q) & 0xffffffff), (fu - q) & 0xffffffff)
    assert np.array_equal(c, f % q)
    # coef_bad(e) == !coef_ok(balanced(e))
    bad = ((e - 32767) & 0xffffffff < 4) | (e == 32640)
    ok = (np.abs(bal) <= 32766) & (bal != 32640)
    assert np.array_equal(bad, ~ok)
