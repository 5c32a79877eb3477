"""File-level integration (the pattern of QuadIron's scripts/test_ec.sh:55-187
driving test/ec_driver.cpp:104-286), on the product through its C++ stream
API: build/qi_ec_driver (tests/host/qi_ec_driver.cpp) encodes k data files
into coding files + text .props files (src/property.cpp:37-78), fragments and
their .props are deleted, the driver repairs the data through
decode_streams_vertical and re-creates every coding file; the repaired data
AND the regenerated codings must equal the originals byte for byte.  Beyond
the reference's md5 check, the first coding files and .props are compared
with the oracle's encode of the same data (parity of the stream path, not
only self-consistency).  Run with -m gpu (the driver needs a HIP device)."""
import os
import subprocess

import numpy as np
import pytest

from qi_testlib import (ROOT, check_windows_vs_oracle, chunk_windows,
                        craft_oor_columns, oracle_encode_blocks)

pytestmark = pytest.mark.gpu

DRIVER = os.path.join(ROOT, "build", "qi_ec_driver")

# (n_data, n_coding, data_loss, coding_loss): scripts/test_ec.sh:176-185
SCENARIOS = [
    (3, 3, [], []),
    (3, 3, [0, 1], [0]),
    (3, 5, [0, 1], [0]),
    (3, 3, [1, 2], [2]),
    (9, 3, [1, 2], [2]),
    (9, 3, [2, 3], [2]),
    (9, 5, [2, 3, 4], [2, 3]),
    (9, 5, [1, 3, 5], [1, 3]),
    (9, 5, [1, 3, 5, 7, 8], []),
    (9, 5, [], [0, 1, 2, 3, 4]),
]


def _name(prefix, kind, zpad, i, ext=""):
    return f"{prefix}.{kind}{i:0{zpad}d}{ext}"


def _run(args, cwd):
    r = subprocess.run([DRIVER] + args, cwd=cwd, capture_output=True, text=True,
                       timeout=120)
    return r


def _props_text(oor, cnt, i):
    return "".join(f"{int(w)} = 1\n" for w in oor[i, :cnt[i]])


def do_test(tmp, fec_type, k, m, data_loss, coding_loss, bs, seed, craft=0):
    if not os.path.exists(DRIVER):
        pytest.fail(f"{DRIVER} missing: build it (make -C quadiron_amd/csrc)")
    sys_ = fec_type == "rs-fnt-sys"
    base = ["-e", fec_type, "-w", "2", "-n", str(k), "-m", str(m), "-p", "foo"]
    r = _run(base + ["-c", "-t"], tmp)
    typ = r.stdout.strip()
    assert typ == ("SYSTEMATIC" if sys_ else "NON_SYSTEMATIC"), r.stderr
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (k, bs), dtype=np.uint8)
    if craft:
        words = data.view(np.uint16).reshape(k, bs // 2).copy()
        for c0 in range(0, bs // 2, 2 ** 21):  # every 4 MiB stream chunk
            craft_oor_columns(k, m, sys_, words, rng, craft,
                              col_range=(c0, min(bs // 2, c0 + 4096)))
        data = words.view(np.uint8).reshape(k, bs)
    dz = len(str(k - 1)) if k > 1 else 1
    no = m if sys_ else k + m
    cz = len(str(no - 1))
    for i in range(k):
        data[i].tofile(os.path.join(tmp, _name("foo", "d", dz, i)))
    r = _run(base + ["-c"], tmp)
    assert r.returncode == 0, r.stderr
    codings = [np.fromfile(os.path.join(tmp, _name("foo", "c", cz, i)), np.uint8)
               for i in range(no)]
    props = [open(os.path.join(tmp, _name("foo", "c", cz, i, ".props"))).read()
             for i in range(no)]
    # the stream path against the oracle's block encode of the same bytes
    # (outputs are packet-size invariant): whole files when
    # small, else window by window (column independence)
    if bs <= 1 << 20:
        cap = 64 + bs // 512
        o_out, o_oor, o_cnt = oracle_encode_blocks(k, m, sys_, data, cap)
        for i in range(no):
            assert (codings[i] == o_out[i]).all(), f"coding {i} differs from the oracle"
            assert props[i] == _props_text(o_oor, o_cnt, i), f"props {i}"
        if craft:
            assert o_cnt.sum() > 0
    else:
        marks = [[int(ln.split("=")[0]) for ln in p.splitlines()] for p in props]
        assert all(ln.endswith(" = 1") for p in props for ln in p.splitlines())
        cap = max(1, max(len(x) for x in marks))
        oor = np.zeros((no, cap), np.uint32)
        cnt = np.array([len(x) for x in marks], np.uint32)
        for i, x in enumerate(marks):
            oor[i, :len(x)] = x
        assert cnt.sum() > 0
        check_windows_vs_oracle(k, m, sys_, data, np.stack(codings), oor, cnt,
                                chunk_windows(bs // 2))

    def mv(name):
        os.rename(os.path.join(tmp, name), os.path.join(tmp, name + ".1"))

    if not sys_:
        for i in range(k):  # every data file removed (test_ec.sh:104-115)
            mv(_name("foo", "d", dz, i))
        for p in data_loss:
            mv(_name("foo", "c", cz, p))
            mv(_name("foo", "c", cz, p, ".props"))
        for p in coding_loss:
            mv(_name("foo", "c", cz, k + p))
            mv(_name("foo", "c", cz, k + p, ".props"))
    else:
        for p in data_loss:
            mv(_name("foo", "d", dz, p))
        for p in coding_loss:
            mv(_name("foo", "c", cz, p))
            mv(_name("foo", "c", cz, p, ".props"))
    r = _run(base + ["-r"], tmp)
    assert r.returncode == 0, r.stderr
    for i in range(k):
        got = np.fromfile(os.path.join(tmp, _name("foo", "d", dz, i)), np.uint8)
        assert (got == data[i]).all(), f"repaired data {i} mismatch"
    for i in range(no):
        got = np.fromfile(os.path.join(tmp, _name("foo", "c", cz, i)), np.uint8)
        assert (got == codings[i]).all(), f"regenerated coding {i} mismatch"
        assert open(os.path.join(tmp, _name("foo", "c", cz, i, ".props"))).read() \
            == props[i]


@pytest.mark.parametrize("fec_type", ["rs-fnt", "rs-fnt-sys"])
@pytest.mark.parametrize("k,m,data_loss,coding_loss", SCENARIOS)
def test_ec_files(tmp_path, fec_type, k, m, data_loss, coding_loss):
    """scripts/test_ec.sh's rs-fnt_2 / rs-fnt-sys_2 matrix, 51200-byte files
    (its `bs`), with a few OOR-forcing columns so the .props carry marks."""
    do_test(str(tmp_path), fec_type, k, m, data_loss, coding_loss, 51200,
            seed=k * 100 + m + len(data_loss) * 7 + len(coding_loss),
            craft=3)


@pytest.mark.parametrize("fec_type", ["rs-fnt", "rs-fnt-sys"])
def test_ec_files_multi_chunk(tmp_path, fec_type):
    """Files of 3 stream chunks (4 MiB each + a tail) with OOR marks in every
    chunk: the pinned two-slot pipeline's offsets, tail handling and marks."""
    do_test(str(tmp_path), fec_type, 9, 5, [1, 3, 5], [1, 3],
            2 * (4 << 20) + 2 * 123457, seed=77, craft=4)
