"""CPU: the plain-C oracle is pinned against golden vectors produced by the
reference itself (tests/golden/gen_golden.py -> oracle/_ref/libqiref.so),
and against the plain O(n^2) DFT (the reference's own equivalence test,
test/fft_utest.cpp:281-302,374-421)."""
import ctypes as C

import numpy as np
import pytest

from qi_testlib import (Q, check_cabi_scenarios, codec, golden_names, load, oracle,
                        oracle_decode_blocks, oracle_encode_blocks,
                        oracle_nf4_decode_blocks, oracle_nf4_encode_blocks,
                        ptrs, vp)


def naive_dft(x, w):
    n = len(x)
    return np.array([sum(int(x[t]) * pow(w, i * t, Q) for t in range(n)) % Q
                     for i in range(n)], np.uint32)


def test_field_constants():
    o = oracle()
    # roots used by the configs
    assert o.qo_nth_root(8) == 4096
    assert o.qo_nth_root(64) == 8224
    assert o.qo_nth_root(1024) == 19139
    assert o.qo_code_len(3) == 4 and o.qo_code_len(64) == 64
    assert o.qo_code_len(1024) == 1024 and o.qo_code_len(1025) == 2048
    for a in (1, 2, 3, 12345, 65536):
        assert o.qo_mul(a, o.qo_inv(a)) == 1
    assert o.qo_mul(65536, 65536) == 1


@pytest.mark.parametrize("n", [2, 8, 16, 64, 256])
def test_fft_is_dft(n):
    o = oracle()
    rng = np.random.default_rng(n)
    w = o.qo_nth_root(n)
    x = rng.integers(0, Q, n).astype(np.uint32)
    x[0] = 65536
    y = np.zeros(n, np.uint32)
    o.qo_fft(n, n, C.c_uint32(w), vp(x), n, vp(y))
    assert (y == naive_dft(x, w)).all()
    # inverse (unnormalised) gives n * x
    z = np.zeros(n, np.uint32)
    o.qo_fft_inv(n, C.c_uint32(w), vp(y), vp(z))
    assert (z == (x.astype(np.uint64) * n % Q)).all()


@pytest.mark.parametrize("n,k", [(8, 4), (64, 16), (64, 13), (1024, 64)])
def test_fft_zero_padded_replication(n, k):
    """Radix2 with data_len = ceil2(k) (replicated zero padding,
    src/fft_2n.h:269-318) equals the DFT of the zero-padded column."""
    o = oracle()
    rng = np.random.default_rng(k)
    w = o.qo_nth_root(n)
    x = rng.integers(0, 65536, k).astype(np.uint32)
    y = np.zeros(n, np.uint32)
    dl = o.qo_code_len(k)
    o.qo_fft(n, dl, C.c_uint32(w), vp(x), k, vp(y))
    xp = np.zeros(n, np.uint32)
    xp[:k] = x
    if n <= 64:
        assert (y == naive_dft(xp, w)).all()
    else:
        for i in rng.integers(0, n, 16):
            ref = sum(int(x[t]) * pow(w, int(i) * t, Q) for t in range(k)) % Q
            assert y[i] == ref


@pytest.mark.parametrize("name", golden_names("blk_"))
def test_oracle_blocks_vs_reference(name):
    g = load(name)
    k, m, sys_, pkt, B, cap = (int(v) for v in g["params"])
    outs, oor, cnt = oracle_encode_blocks(k, m, sys_, g["data"], cap)
    assert (outs == g["outputs"]).all()
    assert (cnt == g["oor_count"]).all()
    assert (oor == g["oor"]).all()
    for p in range(len(g["missing"])):
        ok, dec = oracle_decode_blocks(k, m, sys_, g["outputs"], g["oor"],
                                       g["oor_count"], g["missing"][p],
                                       g["data"])
        assert ok == 1
        assert (dec == g["decoded"][p]).all()


@pytest.mark.parametrize("name", golden_names("cabi_"))
def test_oracle_cabi_vs_reference(name):
    g = load(name)
    k, m, sys_, B, md = (int(v) for v in g["params"])
    c = codec(k, m, sys_)
    o = oracle()
    assert o.qo_metadata_size(C.c_size_t(B)) == md
    d = [g["data"][i].copy() for i in range(k)]
    p = [np.zeros(md + B, np.uint8) for _ in range(m)]
    wanted = np.ones(c.n_outputs, np.int32)
    assert o.qo_fnt32_encode(C.byref(c), ptrs(d), ptrs(p), vp(wanted),
                             C.c_size_t(B)) == 0
    assert (np.stack(d) == g["enc_data"]).all()
    assert (np.stack(p) == g["enc_parity"]).all()
    for t in range(len(g["missing"])):
        miss = g["missing"][t]
        D = [g["enc_data"][i].copy() if not miss[i]
             else np.zeros(md + B, np.uint8) for i in range(k)]
        P = [g["enc_parity"][i].copy() if not miss[k + i]
             else np.zeros(md + B, np.uint8) for i in range(m)]
        assert o.qo_fnt32_decode(C.byref(c), ptrs(D), ptrs(P), vp(miss),
                                 C.c_size_t(B)) == 0
        assert (np.stack(D) == g["decoded"][t]).all()
        D = [g["enc_data"][i].copy() if not miss[i]
             else np.zeros(md + B, np.uint8) for i in range(k)]
        P = [g["enc_parity"][i].copy() if not miss[k + i]
             else np.zeros(md + B, np.uint8) for i in range(m)]
        dest = int(g["dest"][t])
        assert o.qo_fnt32_reconstruct(C.byref(c), ptrs(D), ptrs(P), vp(miss),
                                      C.c_uint(dest), C.c_size_t(B)) == 0
        assert ((D + P)[dest] == g["reconstructed"][t]).all()


@pytest.mark.parametrize("name", golden_names("cabiscn_"))
def test_oracle_cabi_scenarios_vs_reference(name):
    """The reference's exhaustive C-ABI scenario test
    (test/quadiron_c_utest.cpp:283-309: every 0..m erasure pattern of (3, 3),
    every missing index reconstructed) and a cfg2-shaped (16, 48) fixture
    with fewer-than-m erasures, replayed through the oracle's C glue."""
    g = load(name)
    k, m, sys_, B, md = (int(v) for v in g["params"])
    c = codec(k, m, sys_)
    o = oracle()
    assert o.qo_metadata_size(C.c_size_t(B)) == md
    check_cabi_scenarios(
        g,
        lambda D, P, w, B: o.qo_fnt32_encode(C.byref(c), ptrs(D), ptrs(P),
                                             vp(w), C.c_size_t(B)),
        lambda D, P, mi, B: o.qo_fnt32_decode(C.byref(c), ptrs(D), ptrs(P),
                                              vp(mi), C.c_size_t(B)),
        lambda D, P, mi, d, B: o.qo_fnt32_reconstruct(
            C.byref(c), ptrs(D), ptrs(P), vp(mi), C.c_uint(d),
            C.c_size_t(B)))


@pytest.mark.parametrize("name", golden_names("nf4_"))
def test_oracle_nf4_vs_reference(name):
    """RS-NF4 (src/fec_rs_nf4.h) restated as per-lane RS-FNT + (word,
    component-mask) marks, against RsNf4<T> outputs."""
    g = load(name)
    ws, k, m, pkt, B, cap = (int(v) for v in g["params"])
    outs, oor, flags, cnt = oracle_nf4_encode_blocks(ws, k, m, g["data"], cap)
    assert (outs == g["outputs"]).all()
    assert (cnt == g["oor_count"]).all()
    assert (oor == g["oor"]).all() and (flags == g["flags"]).all()
    for p in range(len(g["missing"])):
        ok, dec = oracle_nf4_decode_blocks(ws, k, m, g["outputs"], g["oor"],
                                           g["flags"], g["oor_count"],
                                           g["missing"][p])
        assert ok == 1
        assert (dec == g["decoded"][p]).all()


def test_oracle_fewer_than_k_fails():
    k, m = 4, 4
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (k, 1024), dtype=np.uint8)
    outs, oor, cnt = oracle_encode_blocks(k, m, 0, data)
    miss = np.zeros(k + m, np.int32)
    miss[:m + 1] = 1
    ok, _ = oracle_decode_blocks(k, m, 0, outs, oor, cnt, miss)
    assert ok == 0
