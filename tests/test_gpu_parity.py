"""GPU parity: the HIP path (through the C-ABIs) against the reference's
golden vectors and the CPU oracle, bit-exact.  Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

from qi_testlib import (Q, check_windows_vs_oracle, chunk_windows, codec,
                        craft_dense_oor, craft_oor_columns, golden_names, load, oracle,
                        oracle_decode_blocks, oracle_encode_blocks)

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


# --------------------------------------------------------------- helpers

def fec_encode(hip_lib, k, m, sys_, data, cap):
    import quadiron_amd as qa
    f = qa.Fec(k, m, sys_)
    no = f.n_outputs
    B = data.shape[1]
    outs = np.zeros((no, B), np.uint8)
    oor = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    rows = [np.ascontiguousarray(data[i]) for i in range(k)]
    rc = hip_lib.qi_fec_encode_blocks(
        f.h, qa.ptr_array(rows), qa.ptr_array([outs[i] for i in range(no)]),
        B, oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
        cap)
    assert rc == 0
    return outs, oor, cnt


def fec_decode(hip_lib, k, m, sys_, outputs, oor, cnt, missing, data):
    import quadiron_amd as qa
    f = qa.Fec(k, m, sys_)
    B = outputs.shape[1]
    dec = [np.zeros(B, np.uint8) if (not sys_ or missing[i]) else
           data[i].copy() for i in range(k)]
    par = [None if missing[(k + i) if sys_ else i] else outputs[i].copy()
           for i in range(f.n_outputs)]
    missing = np.ascontiguousarray(missing, np.int32)
    wanted = np.ones(k, np.int32)
    rc = hip_lib.qi_fec_decode_blocks(
        f.h, qa.ptr_array(dec), qa.ptr_array(par),
        oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
        oor.shape[1], missing.ctypes.data_as(C.c_void_p),
        wanted.ctypes.data_as(C.c_void_p), B)
    return rc, np.stack(dec)


# ------------------------------------------------- golden (reference) tests

@pytest.mark.parametrize("name", golden_names("blk_"))
def test_blocks_vs_reference_golden(hip_lib, name):
    g = load(name)
    k, m, sys_, pkt, B, cap = (int(v) for v in g["params"])
    outs, oor, cnt = fec_encode(hip_lib, k, m, sys_, g["data"], cap)
    assert (outs == g["outputs"]).all()
    assert (cnt == g["oor_count"]).all()
    assert (oor == g["oor"]).all()
    for p in range(len(g["missing"])):
        rc, dec = fec_decode(hip_lib, k, m, sys_, g["outputs"], g["oor"],
                             g["oor_count"], g["missing"][p], g["data"])
        assert rc == 1
        bad = np.argwhere(dec != g["decoded"][p])
        assert len(bad) == 0, (
            f"pattern {p} (missing {np.flatnonzero(g['missing'][p]).tolist()}): "
            f"{len(bad)} bytes differ, rows {np.unique(bad[:, 0]).tolist()}, "
            f"bytes {bad[:8, 1].tolist()} .. {bad[-4:, 1].tolist()}")


@pytest.mark.parametrize("name", golden_names("cabi_"))
def test_cabi_vs_reference_golden(hip_lib, name):
    import quadiron_amd as qa
    g = load(name)
    k, m, sys_, B, md = (int(v) for v in g["params"])
    h = qa.QuadironFnt32(2, k, m, sys_)
    assert h.metadata_size(B) == md
    d = [g["data"][i].copy() for i in range(k)]
    p = [np.zeros(md + B, np.uint8) for _ in range(m)]
    wanted = np.ones(m if sys_ else k + m, np.int32)
    assert h.encode(d, p, wanted, B) == 0
    assert (np.stack(d) == g["enc_data"]).all()
    assert (np.stack(p) == g["enc_parity"]).all()
    for t in range(len(g["missing"])):
        miss = np.ascontiguousarray(g["missing"][t], np.int32)
        D = [g["enc_data"][i].copy() if not miss[i]
             else np.zeros(md + B, np.uint8) for i in range(k)]
        P = [g["enc_parity"][i].copy() if not miss[k + i]
             else np.zeros(md + B, np.uint8) for i in range(m)]
        assert h.decode(D, P, miss, B) == 0
        assert (np.stack(D) == g["decoded"][t]).all()
        D = [g["enc_data"][i].copy() if not miss[i]
             else np.zeros(md + B, np.uint8) for i in range(k)]
        P = [g["enc_parity"][i].copy() if not miss[k + i]
             else np.zeros(md + B, np.uint8) for i in range(m)]
        dest = int(g["dest"][t])
        assert h.reconstruct(D, P, miss, dest, B) == 0
        assert ((D + P)[dest] == g["reconstructed"][t]).all()


@pytest.mark.parametrize("name", golden_names("cabiscn_"))
def test_cabi_scenarios_vs_reference_golden(hip_lib, name):
    """The reference's own exhaustive C-ABI test through quadiron_fnt32_*:
    test/quadiron_c_utest.cpp:283-309 runs every 0..m erasure pattern of
    (3, 3), systematic and not (42 patterns each), encode -> decode ->
    reconstruct of EVERY missing fragment on the same buffers; plus a
    cfg2-shaped (16, 48, 64 KiB + 2) fixture whose patterns miss fewer than
    m fragments (the decoder's first-k choice, src/fec_base.h:1199-1236) and
    reconstruct parities while data fragments are missing too
    (src/quadiron_c.cpp:322-369).  Byte-for-byte, FNT1 headers included,
    against the reference's outputs (tests/golden/gen_golden.py
    `_gen_cabi_scn`)."""
    import quadiron_amd as qa
    from qi_testlib import check_cabi_scenarios
    g = load(name)
    k, m, sys_, B, md = (int(v) for v in g["params"])
    h = qa.QuadironFnt32(2, k, m, sys_)
    assert h.metadata_size(B) == md
    check_cabi_scenarios(g, h.encode, h.decode, h.reconstruct)


@pytest.mark.parametrize("k,m,sys_", [(4, 4, 0), (6, 3, 1)])
def test_cabi_multi_chunk_block_vs_oracle(hip_lib, k, m, sys_):
    """quadiron_fnt32_encode / _decode on a block wider than one pipeline
    chunk (4 MiB per fragment: 3 chunks, ragged last one) run the two-slot
    pinned pipeline; every byte of every fragment -- FNT1 headers with the
    OOR offsets included -- matches the oracle's C glue, OOR columns crafted
    next to each chunk seam, and the decode restores the data."""
    import quadiron_amd as qa
    from qi_testlib import ptrs, vp
    rng = np.random.default_rng(1000 + k)
    words = 2 * 2**21 + 12345
    B = 2 * words
    lanes = rng.integers(0, 65536, (k, words), dtype=np.uint16)
    for c0 in (0, 2**21 - 40, 2 * 2**21 - 40, words - 100):
        _craft(k, m, sys_, lanes, rng, 3, col_range=(c0, min(words, c0 + 80)))
    h = qa.QuadironFnt32(2, k, m, sys_)
    md = h.metadata_size(B)
    c = codec(k, m, sys_)
    o = oracle()

    def frags():
        d = [np.concatenate([np.zeros(md, np.uint8), lanes[i].view(np.uint8)])
             for i in range(k)]
        return d, [np.zeros(md + B, np.uint8) for _ in range(m)]
    d, p = frags()
    wanted = np.ones(m if sys_ else k + m, np.int32)
    assert h.encode(d, p, wanted, B) == 0
    od, op = frags()
    assert o.qo_fnt32_encode(C.byref(c), ptrs(od), ptrs(op),
                             vp(np.ones(c.n_outputs, np.int32)), C.c_size_t(B)) == 0
    for x, y in zip(d + p, od + op):
        assert (x == y).all()
    n_marks = sum(int.from_bytes(bytes(f[4:8]), "big") for f in p)
    assert n_marks >= 3
    miss = np.zeros(k + m, np.int32)  # m erasures, data fragment 0 among them
    miss[[0] + list(rng.choice(np.arange(1, k + m), m - 1, replace=False))] = 1

    def received(src_d, src_p):
        return ([src_d[i].copy() if not miss[i] else np.zeros(md + B, np.uint8)
                 for i in range(k)],
                [src_p[i].copy() if not miss[k + i] else np.zeros(md + B, np.uint8)
                 for i in range(m)])
    D, P = received(d, p)
    assert h.decode(D, P, miss, B) == 0
    OD, OP = received(od, op)
    assert o.qo_fnt32_decode(C.byref(c), ptrs(OD), ptrs(OP), vp(miss),
                             C.c_size_t(B)) == 0
    for x, y in zip(D, OD):
        assert (x == y).all()
    for i in range(k):
        assert (D[i][md:] == lanes[i].view(np.uint8)).all()


def test_cabi_word_size_1_rejected(hip_lib):
    import quadiron_amd as qa
    assert hip_lib.quadiron_fnt32_new(1, 3, 3, 0) is None
    with pytest.raises(ValueError):
        qa.QuadironFnt32(1, 3, 3, 0)


def test_cabi_errors(hip_lib):
    import quadiron_amd as qa
    k, m, B = 4, 2, 4096
    h = qa.QuadironFnt32(2, k, m, 0)
    md = h.metadata_size(B)
    rng = np.random.default_rng(5)
    d = [np.concatenate([np.zeros(md, np.uint8),
                         rng.integers(0, 256, B, dtype=np.uint8)])
         for _ in range(k)]
    p = [np.zeros(md + B, np.uint8) for _ in range(m)]
    assert h.encode(d, p, np.ones(k + m, np.int32), B) == 0
    # fewer than k fragments
    miss = np.zeros(k + m, np.int32)
    miss[:m + 1] = 1
    assert h.decode([x.copy() for x in d], [x.copy() for x in p], miss, B) == -1
    # corrupt FNT1 magic of a present fragment
    miss = np.zeros(k + m, np.int32)
    miss[0] = 1
    bad = [x.copy() for x in p]
    bad[0][0] ^= 0xFF
    assert h.decode([x.copy() for x in d], bad, miss, B) == -1


# ------------------------------------------- device batch API vs oracle

_craft = craft_oor_columns


def _batch_roundtrip(k, m, sys_, S, P, seed, n_craft=0, check_oracle=True,
                     encoder=None, oracle_stripes=None, windows=None, ids_fn=None):
    """Encode S random stripes, decode each from its own random k-subset,
    through both decode layouts.  check_oracle: the first 3 stripes' outputs
    and OOR lists bit-exact against the oracle; oracle_stripes + windows:
    those stripes' outputs, OOR lists and decodes against the oracle column
    window by column window (full-size batches); ids_fn(rng, s): stripe s's
    received ids, in the order the caller passes them (default: a sorted
    random k-subset)."""
    torch = _torch()
    import quadiron_amd as qa
    rng = np.random.default_rng(seed)
    plan = qa.Plan(k, m, sys_, encoder=encoder)
    no = plan.n_outputs
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    for s in range(min(S, 2)):
        if n_craft:
            _craft(k, m, sys_, data[s], rng, n_craft)
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((S, no, P), dtype=torch.int16, device="cuda")
    cap = 64 + P // 512
    counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    out_h = out.cpu().numpy().view(np.uint16)
    cnt_h = counts.cpu().numpy().view(np.uint32).reshape(S, no)
    ent_h = entries.cpu().numpy().view(np.uint32).reshape(S, no, cap)
    assert (cnt_h <= cap).all()
    if check_oracle:
        for s in range(min(S, 3)):
            bytes_rows = data[s].view(np.uint8).reshape(k, 2 * P)
            o_out, o_oor, o_cnt = oracle_encode_blocks(k, m, sys_, bytes_rows,
                                                       cap)
            assert (out_h[s].view(np.uint8).reshape(no, 2 * P) == o_out).all()
            assert (cnt_h[s] == o_cnt).all()
            for i in range(no):
                assert (np.sort(ent_h[s, i, :cnt_h[s, i]])
                        == o_oor[i, :o_cnt[i]]).all()
    # decode with a random k-subset per stripe (sys: drop a random data row
    # set so that a real decode happens)
    ids = np.zeros((S, k), np.uint16)
    for s in range(S):
        ids[s] = (ids_fn(rng, s) if ids_fn else
                  np.sort(rng.choice(k + m, k, replace=False)))
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    # a context buffer full of garbage: the context kernel must write every
    # word the decode reads (it skips the tiles' zero halves at k > 32)
    ctx = torch.randint(0, 256, (plan.ctx_bytes(S, P),), dtype=torch.uint8,
                        device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap, h_ids=ids)
    dec = torch.zeros((S, k, P), dtype=torch.int16, device="cuda")
    err = plan.decode(ctx, di, out, dec, data=dd, counts=counts,
                      entries=entries, cap=cap)
    torch.cuda.synchronize()
    assert err == 0
    dec_h = dec.cpu().numpy().view(np.uint16)
    assert (dec_h == data).all()
    # a context from the ids alone (no buckets: init_context_dec before the
    # marks exist); the decode reads the marks from the buckets itself
    ctx3 = torch.randint(0, 256, (plan.ctx_bytes(S, P),), dtype=torch.uint8,
                         device="cuda")
    plan.decode_ctx(di, ctx3, P, h_ids=ids)
    dec3 = torch.zeros_like(dec)
    assert plan.decode(ctx3, di, out, dec3, data=dd, counts=counts,
                       entries=entries, cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec3, dd)
    for s in oracle_stripes or ():
        ent_s = ent_h[s].copy()
        for i in range(no):  # the buckets are unordered; the oracle's ascend
            ent_s[i, :cnt_h[s, i]].sort()
        missing = np.ones(k + m, np.int32)
        missing[ids[s].astype(np.int64)] = 0
        check_windows_vs_oracle(
            k, m, sys_, data[s].view(np.uint8).reshape(k, 2 * P),
            out_h[s].view(np.uint8).reshape(no, 2 * P), ent_s, cnt_h[s],
            windows, missing, dec_h[s].view(np.uint8).reshape(k, 2 * P))

    # the packed staging layout (qi_gpu_decode_packed): received rows back
    # to back in id order, OOR buckets by position
    idx = torch.from_numpy(ids.astype(np.int64)).cuda()
    if sys_:
        full = torch.cat([dd, out], dim=1)
        zc = torch.zeros((S, k), dtype=torch.int32, device="cuda")
        fcnt = torch.cat([zc, counts.view(S, no)], dim=1)
        fent = torch.cat([torch.zeros((S, k, cap), dtype=torch.int32,
                                      device="cuda"),
                          entries.view(S, no, cap)], dim=1)
    else:
        full, fcnt, fent = out, counts.view(S, no), entries.view(S, no, cap)
    recv = torch.gather(full, 1, idx[:, :, None].expand(S, k, P)).contiguous()
    pcnt = torch.gather(fcnt, 1, idx).contiguous()
    pent = torch.gather(fent, 1, idx[:, :, None].expand(S, k, cap)).contiguous()
    ctx2 = torch.full_like(ctx, 0xA5)
    plan.decode_ctx_packed(di, ctx2, P, pcnt, pent, cap, h_ids=ids)
    dec2 = torch.zeros_like(dec)
    assert plan.decode_packed(ctx2, recv, dec2, pcnt, pent, cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec2, dd)
    return plan


@pytest.mark.parametrize("k,m,sys_,S,P", [
    (4, 4, 0, 100, 512),      # cfg1 shape
    (16, 48, 0, 8, 4096),     # cfg2 shape, small P
    (16, 48, 0, 3, 4093),     # ragged P (tail columns)
    (16, 48, 1, 4, 2048),     # systematic
    (3, 3, 0, 5, 1000),
    (9, 5, 1, 5, 999),
    (1, 1, 0, 2, 300),
    (7, 1, 1, 2, 300),
    (32, 32, 0, 2, 1024),
    (33, 31, 0, 2, 513),      # K = 64 codelet, k not a power of two
    (64, 960, 0, 2, 2048),    # cfg3 shape
    # 64 < k <= 128: matrix cores at KS = 8 (whole 1024-column tiles) and
    # the dot2 kernel at KP = 64 (column tails)
    (65, 63, 0, 2, 300),
    (65, 63, 0, 2, 1024),
    (100, 28, 0, 2, 1000),
    (100, 28, 0, 3, 2148),
    (100, 50, 1, 2, 999),
    (100, 50, 1, 2, 2048),    # systematic: generator + mode-1 contexts
    (128, 128, 0, 2, 2048),
    (128, 100, 1, 1, 1100),
    # 128 < k <= 256: matrix cores at KS = 16 (D2 folded in the epilogue),
    # the context's matrix rows in global memory, dot2 tails at KP = 128
    (200, 56, 0, 3, 1000),    # quadiron_fnt32_new(2, 200, 56, ...)
    (200, 56, 0, 2, 2112),
    (200, 56, 1, 2, 513),
    (200, 56, 1, 2, 1024),
    (256, 768, 0, 2, 700),
    (256, 768, 0, 1, 2048),
    (129, 127, 1, 1, 1100),
    (130, 900, 1, 1, 300),
    # 256 < k <= 384 with whole 1024-column tiles: the operand-stationary
    # matrix kernel at KS = 20 / 24 (k x k contexts, the generator encode)
    (300, 212, 0, 2, 1024),
    (257, 255, 0, 1, 2048),
    (320, 100, 1, 2, 1024),   # systematic: generator + mode-1 contexts
    (321, 63, 0, 2, 1024),    # KS = 24
    (384, 128, 0, 1, 2048),   # largest generator / systematic matrix-path k
    (384, 100, 1, 1, 1024),
    # 384 < k <= 640, n - k > 64, whole 1024-column tiles: the decode on the
    # matrix cores at KS = 40 in two K chunks (round 6; the encode stays on
    # the NTT engine); systematic: the two source regions, the mode-1
    # contexts' rows through global memory
    (385, 127, 0, 2, 1024),   # smallest KS = 40 code
    (500, 524, 0, 1, 2048),
    (600, 1400, 0, 1, 1024),  # the k600 bench code
    (640, 384, 0, 1, 1024),   # largest matrix-path k
    (385, 127, 1, 2, 1024),
    (600, 1400, 1, 1, 1024),
    (640, 384, 1, 1, 2048),
    # systematic generators between 2^18 and 2^20 entries (round 6: the
    # closed-form Lagrange rows made them cheap to build)
    (300, 1000, 1, 1, 1024),  # KS = 20, 1000 x 300
    (640, 1600, 1, 1, 1024),  # KS = 40, 1600 x 640 (n = 4096)
    # k > 256: the NTT-structured general path (ntt.hip)
    (257, 255, 0, 1, 300),    # smallest NTT-path code
    (300, 100, 1, 1, 300),    # systematic: interpolation + NTT_n encode
    (1000, 24, 0, 1, 260),    # len_2k = 2048 > n = 1024
    # the LDS engine's 16-byte row pieces (P % 8 == 0) and table placements:
    # decode with ids / inv_A in the image rows INTT_n leaves free (n < nmax),
    # tables from global memory (sys decode; n = nmax), tables staged
    (1000, 24, 0, 2, 1024),
    (1000, 24, 1, 1, 512),
    (600, 1400, 0, 1, 256),   # n = len_2k = 2048: no free image rows
    (385, 127, 0, 2, 1032),   # smallest k past the matrix path
    # few erasures (n - k <= 64): the erasure decode (and the systematic
    # encode as the same solve): n = 512 / 1024 / 2048, e = 4 .. 64
    (450, 62, 0, 2, 1024),
    (448, 64, 1, 2, 1000),
    (500, 12, 1, 2, 1000),
    (1020, 4, 0, 2, 333),
    (2000, 48, 0, 1, 520),    # len_2k = 4096: encode on the multi-pass engine
    (1990, 58, 1, 1, 256),
])
def test_batch_vs_oracle(k, m, sys_, S, P):
    _batch_roundtrip(k, m, sys_, S, P, seed=k * 1000 + m + P, n_craft=16)


def _random_shapes(n, seed):
    """n codes drawn from a fixed seed: k near every routing boundary (the
    matrix-core K-steps, the context kernels, the NTT engine) or uniform up
    to 700, m small (erasure decode), medium, large or very large (n up to
    16384: the multi-pass engine), ragged and whole-tile widths, both code
    types."""
    rng = np.random.default_rng(seed)
    edges = [1, 2, 3, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 255, 256,
             257, 319, 320, 321, 383, 384, 385, 639, 640, 641, 1000]
    shapes = []
    while len(shapes) < n:
        k = int(rng.choice(edges)) if rng.random() < 0.6 else int(rng.integers(1, 700))
        kind = int(rng.integers(4))
        m = (int(rng.integers(1, 65)) if kind == 0 else
             int(rng.integers(1, 400)) if kind == 1 else
             int(rng.integers(400, 3000)) if kind == 2 else int(rng.integers(3000, 12000)))
        if k + m > 16384:
            continue
        P = int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 1200)), 1024, 2048]))
        shapes.append((k, m, int(rng.integers(2)), int(rng.integers(1, 4)), P))
    return shapes


@pytest.mark.parametrize("k,m,sys_,S,P", _random_shapes(64, 20261019))
def test_random_shapes_vs_oracle(k, m, sys_, S, P):
    """A seeded sweep beyond the hand-picked shapes above: encode outputs and
    OOR lists of the first stripes bit-exact against the oracle, every
    stripe decoded back from its own random k-subset (both layouts), OOR
    columns crafted into the data."""
    _batch_roundtrip(k, m, sys_, S, P, seed=7 * k + 13 * m + P + sys_, n_craft=8)


@pytest.mark.parametrize("k,m,sys_,S,P", [
    (16, 48, 1, 6, 2048),     # KS = 1: matrix_mfma_kernel, LDS context
    (64, 960, 1, 6, 2048),    # matrix_os_kernel<4, ...>, LDS context
    (200, 56, 1, 6, 1024),    # k > 128 context, KS = 16 at two row blocks per wave
    (200, 56, 1, 6, 1000),    # the same with dot2 column tails
    (300, 212, 1, 6, 1024),   # KS = 20
    (600, 1400, 1, 6, 1024),  # KS = 40, two K chunks
    (64, 960, 0, 4, 2048),    # non-systematic: any order, nothing reordered
    (600, 1400, 0, 4, 1024),
])
def test_decode_ids_any_order(k, m, sys_, S, P):
    """Received ids in any order.  The systematic decode contexts list the
    received fragments region by region (data first: ctx.hip order_ids), and
    the two-region matrix kernel loads each row once through its region's
    descriptor, with one extra load for the pass that straddles the
    boundary; the route entries and the ids the decode reads follow the same
    order.  Stripes: every data fragment received (shuffled), only parity
    (m >= k), one data fragment among parity, then shuffled random
    subsets; OOR columns crafted into the first two stripes' data."""
    def ids_fn(rng, s):
        if s == 0:
            sel = np.arange(k)
        elif s == 1 and m >= k:
            sel = k + rng.choice(m, k, replace=False)
        elif s == 2 and m >= k - 1:
            sel = np.concatenate([[rng.integers(k)], k + rng.choice(m, k - 1, replace=False)])
        else:
            sel = rng.choice(k + m, k, replace=False)
        return rng.permutation(sel)
    _batch_roundtrip(k, m, sys_, S, P, seed=31 * k + m + P + sys_, n_craft=16, ids_fn=ids_fn)


def _slice_windows(P, W=4096, width=256):
    """Column windows of a P-word block: the start, every multi-pass column
    slice seam (slices of W words) and the tail."""
    wins = {(0, min(P, width)), (max(0, P - width), P)}
    for c in range(W, P, W):
        wins.add((max(0, c - width // 2), min(P, c + width // 2)))
    return sorted(wins)


@pytest.mark.parametrize("k,m,sys_,S,P,stripes", [
    (300, 16000, 0, 1, 4500, [0]),         # n = 16384: columns in 2 slices
    (300, 3000, 0, 70, 256, [0, 63, 64, 69]),  # n = 4096: 2 stripe groups
    (260, 200, 0, 600, 256, [0, 299, 599]),    # LDS engine, 600 x 8 tiles
    (260, 16000, 1, 1, 4200, [0]),         # systematic, sliced
    (1100, 100, 0, 3, 700, [0, 2]),        # len_2k = 4096 > n = 2048
    (130, 16000, 0, 1, 4500, [0]),         # matrix path: 16130 x 130 generator
])
def test_general_path_slicing(k, m, sys_, S, P, stripes):
    """The general path's multi-pass engine (max(n, len_2k) > 2048) cuts a
    batch into column slices and stripe groups (HBM scratch budget).  Every
    output row, OOR list and decoded row of the checked stripes is compared
    with the oracle (pinned to the reference by the blk_k300_m3796,
    blk_k260_m3000_sys, blk_k1100_m100 and blk_k300_m16000 fixtures), window
    by window around each slice seam, plus a round trip of every stripe."""
    torch = _torch()
    import quadiron_amd as qa
    rng = np.random.default_rng(k + m + S)
    plan = qa.Plan(k, m, sys_)
    no = plan.n_outputs
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    for s in stripes:
        _craft(k, m, sys_, data[s], rng, 6)
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((S, no, P), dtype=torch.int16, device="cuda")
    cap = 64 + P // 64
    counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    cnt_h = counts.cpu().numpy().view(np.uint32).reshape(S, no)
    ent_h = entries.cpu().numpy().view(np.uint32).reshape(S, no, cap).copy()
    assert (cnt_h <= cap).all()
    for s in stripes:  # the buckets are unordered; the oracle's lists ascend
        for i in range(no):
            ent_h[s, i, :cnt_h[s, i]].sort()
    ids = np.zeros((S, k), np.uint16)
    for s in range(S):
        ids[s] = np.sort(rng.choice(k + m, k, replace=False))
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap)
    dec = torch.zeros((S, k, P), dtype=torch.int16, device="cuda")
    assert plan.decode(ctx, di, out, dec, data=dd, counts=counts,
                       entries=entries, cap=cap) == 0
    assert torch.equal(dec, dd)
    out_h = out.cpu().numpy().view(np.uint16)
    dec_h = dec.cpu().numpy().view(np.uint16)
    wins = _slice_windows(P)
    for s in stripes:
        missing = np.ones(k + m, np.int32)
        missing[ids[s].astype(np.int64)] = 0
        check_windows_vs_oracle(
            k, m, sys_, data[s].view(np.uint8).reshape(k, 2 * P),
            out_h[s].view(np.uint8).reshape(no, 2 * P), ent_h[s], cnt_h[s],
            wins, missing, dec_h[s].view(np.uint8).reshape(k, 2 * P))


@pytest.mark.parametrize("k,m,S,P", [
    (16, 48, 3, 4096),        # 64 x 16 generator, KS = 1
    (33, 31, 2, 2048),        # KS = 4 with padded inputs (x64 MFMA, zero K halves)
    (64, 960, 2, 2048),       # cfg3 generator, row blocks split over waves
])
def test_matrix_encode_flag_vs_oracle(k, m, S, P):
    """QI_PLAN_ENC_MATRIX sends non-systematic encodes through the
    matrix-core kernel (the default at K = 64 only): bit-exact on every
    generator shape, including the permuted rows of the cfg3 Vandermonde
    generator."""
    _batch_roundtrip(k, m, 0, S, P, seed=7 * k + m + P, n_craft=16, encoder="matrix")


@pytest.mark.parametrize("k,m,S,P", [
    (64, 960, 2, 2048),       # cfg3 shape: the 64-point codelet kernel
    (33, 31, 2, 513),
])
def test_codelet_encode_flag_vs_oracle(k, m, S, P):
    """QI_PLAN_ENC_CODELETS keeps the register FNT codelets at K = 64 too."""
    _batch_roundtrip(k, m, 0, S, P, seed=11 * k + m + P, n_craft=16,
                     encoder="codelets")


def _spread(S, step=8):
    """First, last and every `step`-th stripe of a batch."""
    return sorted(set(range(0, S, step)) | {S - 1})


def test_cfg2_full_size_roundtrip():
    """BASELINE cfg2 geometry (k=16, n=64, 64 KiB packets) at 32 stripes:
    encode -> per-stripe random erasures -> decode == data; stripes 0-2
    bit-exact against the oracle over the whole block, and the first, last
    and every 8th stripe by column windows (start, middle, end) with their
    OOR lists and decodes."""
    P = 32768
    _batch_roundtrip(16, 48, 0, 32, P, seed=2, n_craft=8, check_oracle=True,
                     oracle_stripes=_spread(32),
                     windows=[(0, 512), (P // 2 - 256, P // 2 + 256), (P - 512, P)])


def test_cfg4_all_patterns_distinct():
    """cfg4: per-stripe n-k random erasures (every stripe its own context);
    the first, last and every 8th stripe's outputs, OOR lists and decodes
    against the oracle over the whole block."""
    P = 2048
    _batch_roundtrip(16, 48, 0, 256, P, seed=4, n_craft=0, check_oracle=False,
                     oracle_stripes=_spread(256), windows=[(0, P)])


def test_cfg3_random_patterns_vs_oracle():
    """cfg3 geometry (k=64, n=1024, 4 KiB packets) at 96 stripes, each
    decoded from its own random 64-subset of the 1024 fragments: the first,
    last and every 8th stripe against the oracle by column windows."""
    P = 2048
    _batch_roundtrip(64, 960, 0, 96, P, seed=6, n_craft=0, check_oracle=False,
                     oracle_stripes=_spread(96),
                     windows=[(0, 256), (1024 - 128, 1024 + 128), (P - 256, P)])


def test_cfg3_full_batch_vs_oracle():
    """BASELINE configs[2] at its full bench size: 1024 stripes of k=64,
    n=1024, 4 KiB packets, each decoded from its own random 64-subset (the
    bench's batch checks only the round trip); every stripe round-trips, and
    stripes 0, 32, 64, ..., 1023 match the oracle by column windows
    (outputs, OOR lists, decodes)."""
    P = 2048
    _batch_roundtrip(64, 960, 0, 1024, P, seed=7, n_craft=0, check_oracle=False,
                     oracle_stripes=_spread(1024, 32),
                     windows=[(0, 128), (1024 - 64, 1024 + 64), (P - 128, P)])


def test_cfg2_full_batch_vs_oracle():
    """BASELINE configs[1] at its full bench size: 4096 stripes of k=16,
    n=64, 64 KiB packets (4 GiB of data, 16 GiB coded), each decoded from its
    own random 16-subset (the bench checks only the round trip):
    every stripe round-trips through both decode layouts, and stripes 0, 128,
    256, ..., 4095 match the oracle by column windows at the start, the
    middle and the end of the packet (outputs, OOR lists, decodes)."""
    P = 32768
    _batch_roundtrip(16, 48, 0, 4096, P, seed=8, n_craft=8, check_oracle=False,
                     oracle_stripes=_spread(4096, 128),
                     windows=[(0, 128), (P // 2 - 64, P // 2 + 64), (P - 128, P)])


@pytest.mark.parametrize("k,m,S,P", [
    (16, 48, 4096, 256),    # ~0.1 % of the stripes need a row scale
    (64, 960, 96, 1024),    # ~27 %
    (100, 28, 48, 1024),    # KS = 8
    (128, 128, 24, 1024),
    (200, 56, 24, 1024),    # the BIG context packed straight into the tiles
    (256, 768, 8, 2048),
])
def test_decode_row_scales_many_stripes(k, m, S, P):
    """Many random erasure patterns: the decode contexts whose interpolation
    rows hold an entry neither kernel can take (balanced |c| > 32766 or
    32640) are rescaled by a unit s on the GPU (pack_row's search); every
    stripe must still decode back to its data."""
    _batch_roundtrip(k, m, 0, S, P, seed=3 * k + S, n_craft=0, check_oracle=False)


@pytest.mark.parametrize("k,m,sys_", [
    (300, 100, 0), (300, 100, 1),   # 256 < k <= 384: the NTT engine takes them
    (500, 524, 0), (500, 524, 1),   # 384 < k <= 640 (KS = 40 plans): the same
    (16, 48, 0), (64, 960, 0), (200, 56, 1),  # the dot2 kernel, its context
                                              # sections filled from the tiles
])
def test_unaligned_rows_whole_tiles(k, m, sys_):
    """A whole-tile width (1024 columns) with rows the matrix cores cannot
    address (base offset by one u16, odd row strides).  256 < k <= 384: the
    encode runs the NTT engine and the decode the NTT context kept behind the
    matrix one (these calls used to fail with -3).  k <= 256: the
    context was built with the matrix-core form only (whole tiles), and the
    decode fills the dot2 kernel's sections from the operand tiles first.
    Then the same contexts decode aligned copies on the matrix cores."""
    torch = _torch()
    import quadiron_amd as qa
    S, P = 2, 1024
    rng = np.random.default_rng(k + 300 + sys_)
    plan = qa.Plan(k, m, sys_)
    no = plan.n_outputs
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    _craft(k, m, sys_, data[0], rng, 8)
    dbig = torch.zeros((S, k, P + 1), dtype=torch.int16, device="cuda")
    dd = dbig[:, :, 1:]
    dd.copy_(torch.from_numpy(data.view(np.int16)))
    obig = torch.zeros((S, no, P + 3), dtype=torch.int16, device="cuda")
    out = obig[:, :, 3:]
    cap = 64
    counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    out_h = out.cpu().numpy().view(np.uint16)
    cnt_h = counts.cpu().numpy().view(np.uint32).reshape(S, no)
    ent_h = entries.cpu().numpy().view(np.uint32).reshape(S, no, cap)
    o_out, o_oor, o_cnt = oracle_encode_blocks(
        k, m, sys_, data[0].view(np.uint8).reshape(k, 2 * P), cap)
    assert (out_h[0].view(np.uint8).reshape(no, 2 * P) == o_out).all()
    assert (cnt_h[0] == o_cnt).all() and cnt_h[0].sum() > 0
    for i in range(no):
        assert (np.sort(ent_h[0, i, :cnt_h[0, i]]) == o_oor[i, :o_cnt[i]]).all()
    # stripe 1's ids shuffled: the lazily built sections follow the order
    # the context lists them in (systematic: data fragments first)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) if s == 0 else
                    rng.permutation(rng.choice(k + m, k, replace=False)) for s in range(S)])
    ids = ids.astype(np.uint16)
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.randint(0, 256, (plan.ctx_bytes(S, P),), dtype=torch.uint8,
                        device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap)
    decbig = torch.zeros((S, k, P + 1), dtype=torch.int16, device="cuda")
    dec = decbig[:, :, 1:]
    assert plan.decode(ctx, di, out, dec, data=dd, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)
    # the same contexts with aligned copies of the rows: the matrix cores
    out2 = out.contiguous()
    dec2 = torch.zeros((S, k, P), dtype=torch.int16, device="cuda")
    assert plan.decode(ctx, di, out2, dec2, data=dd.contiguous(), counts=counts,
                       entries=entries, cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec2, dd)
    # a second unaligned decode reuses the sections the first one filled
    # (the context's lazy word)
    dec.zero_()
    assert plan.decode(ctx, di, out, dec, data=dd, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)
    # other patterns built into the same buffer: the builder clears the lazy
    # word, so the next unaligned decode fills the sections again
    ids2 = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
    di2 = torch.from_numpy(ids2.astype(np.uint16).view(np.int16)).cuda()
    plan.decode_ctx(di2, ctx, P, counts, entries, cap)
    dec.zero_()
    assert plan.decode(ctx, di2, out, dec, data=dd, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)


def test_lazy_ntt_ctx_two_streams():
    """256 < k <= 384 at whole tiles: the context holds the matrix form, and
    the NTT engine's half is built by the first decode whose rows the matrix
    cores cannot address.  Two such decodes from ONE context on two streams
    at once may both find that half unbuilt and both build it; every word of
    it is written once with its final value (no transient -1 in the position
    map), so both decodes come out right.  Repeated over fresh
    contexts (each rebuild clears the lazy word)."""
    torch = _torch()
    import quadiron_amd as qa
    k, m, S, P = 300, 212, 4, 1024
    plan = qa.Plan(k, m, False)
    rng = np.random.default_rng(23)
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    obig = torch.zeros((S, plan.n_outputs, P + 1), dtype=torch.int16, device="cuda")
    out = obig[:, :, 1:]  # rows at odd u16 offsets: the NTT engine decodes
    cap = 64
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(4):
        ids = np.stack([np.sort(rng.choice(k + m, k, replace=False))
                        for _ in range(S)]).astype(np.uint16)
        di = torch.from_numpy(ids.view(np.int16)).cuda()
        plan.decode_ctx(di, ctx, P, counts, entries, cap)
        torch.cuda.synchronize()
        decs = [torch.zeros((S, k, P + 1), dtype=torch.int16, device="cuda")[:, :, 1:]
                for _ in range(2)]
        for st, dec in zip((s1, s2), decs):
            assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                               cap=cap, stream=st.cuda_stream, check=False) == 0
        torch.cuda.synchronize()
        assert plan.take_error() == 0
        for dec in decs:
            assert torch.equal(dec, dd), rep


def test_big_matrix_ctx_sized_for_a_wider_batch():
    """A context buffer sized for the widest batch (ragged: NTT format) holds
    the contexts of a narrower whole-tile batch (matrix format, larger): the
    size query is a bound over every width up to the one asked (ADVICE r3:
    the matrix context overflowed the buffer).  Guard bytes behind the
    buffer must stay untouched."""
    torch = _torch()
    import quadiron_amd as qa
    k, m, S, Pmax, P = 300, 212, 2, 1500, 1024
    plan = qa.Plan(k, m, False)
    assert plan.ctx_bytes(S, Pmax) >= plan.ctx_bytes(S, P)
    rng = np.random.default_rng(17)
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((S, plan.n_outputs, P), dtype=torch.int16, device="cuda")
    cap = 64
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False))
                    for _ in range(S)]).astype(np.uint16)
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    nb = plan.ctx_bytes(S, Pmax)
    buf = torch.full((nb + 4096,), 0x5A, dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, buf[:nb], P, counts, entries, cap)
    dec = torch.zeros_like(dd)
    assert plan.decode(buf[:nb], di, out, dec, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)
    assert bool((buf[nb:] == 0x5A).all())


def test_empty_and_tiny_blocks(hip_lib):
    for B in (0, 1, 2, 3, 130):
        k, m = 3, 2
        data = np.random.default_rng(B).integers(0, 256, (k, B),
                                                 dtype=np.uint8)
        outs, oor, cnt = fec_encode(hip_lib, k, m, 0, data, 64)
        o_out, o_oor, o_cnt = oracle_encode_blocks(k, m, 0, data, 64)
        assert (outs == o_out).all() and (cnt == o_cnt).all()


@pytest.mark.parametrize("k,m", [(16, 48), (32, 32)])
def test_dense_oor_tile_uses_bucket_scan(k, m):
    """More than kRouteCap (15) marks of received rows inside one 1024-column
    tile: the decode falls back from the context's route table to scanning
    the OOR buckets; output still bit-exact (k=16: dot2 kernel, k=32: the
    matrix-core kernel)."""
    torch = _torch()
    import quadiron_amd as qa
    S, P = 1, 2048
    rng = np.random.default_rng(99)
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    _craft(k, m, 0, data[0], rng, 200, rows=range(k), col_range=(512, 1024))
    plan = qa.Plan(k, m, False)
    no = plan.n_outputs
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((S, no, P), dtype=torch.int16, device="cuda")
    cap = 512
    counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    ids = np.arange(k, dtype=np.uint16)[None, :]
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap)
    dec = torch.zeros_like(dd)
    assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    cnt = counts.cpu().numpy()[:k]
    assert cnt.sum() > 100, cnt
    assert torch.equal(dec, dd)


def _dense_tile_setup(k, m, n_marks, P=2048, seed=99):
    """Data whose encoding has ~n_marks OOR marks on the received rows
    0..k-1 inside the first 1024-column tile."""
    torch = _torch()
    import quadiron_amd as qa
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 65536, (1, k, P), dtype=np.uint16)
    _craft(k, m, 0, data[0], rng, n_marks, rows=range(k), col_range=(0, 1024))
    plan = qa.Plan(k, m, False)
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((1, plan.n_outputs, P), dtype=torch.int16, device="cuda")
    return plan, dd, out, P


@pytest.mark.parametrize("k,m", [(16, 48), (32, 32)])
def test_dense_tile_over_scratch_decodes(k, m):
    """More than kMaxTileOor (256) marks of the received rows in ONE column
    tile: the reference has no such limit, and neither does the decode --
    the tile takes the slow path (matrix_redo_kernel) instead of failing
    (k=16: matrix cores KS=1, k=32: KS=2, 1024- and 512-column blocks)."""
    torch = _torch()
    plan, dd, out, P = _dense_tile_setup(k, m, 600)
    cap = 1024
    no = plan.n_outputs
    counts = torch.zeros(no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    cnt = counts.cpu().numpy()
    assert cnt[:k].sum() > 300, cnt[:k]
    assert cnt.max() <= cap
    ids = np.arange(k, dtype=np.uint16)[None, :]
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(1, P), dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap, h_ids=ids)
    dec = torch.zeros_like(dd)
    assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)


@pytest.mark.parametrize("k,m,per_col,ranges,P", [
    # KS = 8 (256-column blocks): 2 marks per column over 4 blocks
    (100, 28, 2, [(0, 1024)], 2048),
    # KS = 16 (64-column blocks): 5 per column over 12 blocks -- more slow
    # tiles than a 256-column-grain list held -- plus the dot2 tail
    # (KP = 128, 256-column tiles) past the last whole 1024-column tile
    (200, 56, 5, [(0, 768), (2048, 2348)], 2348),
    (256, 768, 5, [(64, 832)], 2048),
    # 256 < k <= 384, whole tiles: the operand-stationary kernel at KS = 20
    (300, 100, 5, [(0, 768)], 1024),
    # 384 < k <= 640, whole tiles: KS = 40 in two K chunks (the redo's
    # scratch for 400 inputs in the kernel's LDS)
    (400, 100, 5, [(0, 768)], 1024),
    # k > 256, ragged width: the NTT engine walks the buckets itself (no
    # tile list)
    (300, 100, 5, [(0, 768)], 1000),
])
def test_dense_tiles_spread_decode(k, m, per_col, ranges, P):
    """Several OOR marks in every column of many tiles (crafted by solving
    for per_col data rows): every tile overflows the kernels' LDS mark list,
    the slow-tile list holds one entry per tile of the narrowest block
    width (a 256-column-grain list overflowed into the next
    stripe's context at KS = 16) and the redo restores every mark; two
    stripes so an overflow into the neighbour would show."""
    torch = _torch()
    import quadiron_amd as qa
    rng = np.random.default_rng(k + per_col)
    S = 2
    data = rng.integers(0, 65536, (S, k, P), dtype=np.uint16)
    crafted = 0
    for lo, hi in ranges:
        crafted += craft_dense_oor(k, m, data[0], rng, range(lo, hi), range(k),
                                   per_col)
    assert crafted > 0.8 * sum(hi - lo for lo, hi in ranges)
    plan = qa.Plan(k, m, False)
    no = plan.n_outputs
    dd = torch.from_numpy(data.view(np.int16)).cuda()
    out = torch.zeros((S, no, P), dtype=torch.int16, device="cuda")
    cap = 1024
    counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    cnt = counts.cpu().numpy().reshape(S, no)
    assert cnt.max() <= cap
    assert cnt[0, :k].sum() >= per_col * crafted
    ids = np.tile(np.arange(k, dtype=np.uint16), (S, 1))
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.randint(0, 256, (plan.ctx_bytes(S, P),), dtype=torch.uint8,
                        device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap, h_ids=ids)
    dec = torch.zeros_like(dd)
    assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)
    assert plan.take_error() == 0
    # the same context serves a second decode (the redo emptied its lists)
    dec.zero_()
    assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                       cap=cap) == 0
    torch.cuda.synchronize()
    assert torch.equal(dec, dd)


@pytest.mark.parametrize("k,m", [(16, 48), (100, 28), (200, 56), (300, 100), (400, 100)])
def test_decode_bucket_overflow_raises(k, m):
    """A decode reading an OOR bucket whose count exceeds its capacity lost
    marks: it must raise the plan's sticky error, not return wrong data
    silently (the reference returns -1 on header overflow,
    src/property.h:106-108).  k = 16, 100, 200: matrix cores at KS = 1, 8,
    16; k = 300, 400: the operand-stationary kernel at KS = 20 / 40."""
    torch = _torch()
    plan, dd, out, P = _dense_tile_setup(k, m, 200, seed=5)
    cap = 2
    no = plan.n_outputs
    counts = torch.zeros(no, dtype=torch.int32, device="cuda")
    entries = torch.zeros(no * cap, dtype=torch.int32, device="cuda")
    plan.encode(dd, out, counts, entries, cap)
    torch.cuda.synchronize()
    assert counts.cpu().numpy()[:k].max() > cap  # exact counts past cap
    assert plan.take_error() == 0
    ids = np.arange(k, dtype=np.uint16)[None, :]
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(1, P), dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, ctx, P, counts, entries, cap, h_ids=ids)
    dec = torch.zeros_like(dd)
    assert plan.decode(ctx, di, out, dec, counts=counts, entries=entries,
                       cap=cap) != 0
    assert plan.take_error() == 0  # reset by reading


@pytest.mark.parametrize("bad", ["repeated", "past_n"])
@pytest.mark.parametrize("k,m,n,P,kern", [
    (500, 10, 512, 64, "ntt_eras_kernel"),          # erasure context
    (16, 48, 64, 64, "decode_ctx_lds_kernel<128>"),  # matrix contexts
    (64, 960, 1024, 1024, "decode_ctx_lds_kernel<256>"),
    (200, 56, 256, 1024, "decode_ctx_kernel<1024, true>"),
    (300, 212, 512, 1024, "decode_ctx_kernel<1024, true>"),
    (600, 1400, 2048, 256, "ntt_ctx_kernel"),       # the general NTT decode
])
def test_ctx_bad_ids_raise(bad, k, m, n, P, kern):
    """Every decode-context builder checks the received ids: a repeated id
    (two equal points: A'(x_i) = 0, or more than n - k positions looking
    erased) or an id >= n must raise the plan's sticky error and write
    nothing outside the stripe's own context: the next stripe's context is
    the one it builds alone, and guard bytes behind the buffer stay
    untouched (the erasure context; r5: the matrix contexts)."""
    torch = _torch()
    import quadiron_amd as qa
    S = 2
    plan = qa.Plan(k, m, False)
    assert kern in plan.kernels(P)
    rng = np.random.default_rng(3)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False))
                    for _ in range(S)]).astype(np.uint16)
    if bad == "repeated":
        ids[0, 7] = ids[0, 6]
    else:
        ids[0, -1] = n + 88
    di = torch.from_numpy(ids.view(np.int16)).cuda()
    nb = plan.ctx_bytes(S, P)
    cs = plan.ctx_bytes(1, P)
    buf = torch.full((nb + 4096,), 0x5A, dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di, buf[:nb], P)
    torch.cuda.synchronize()
    assert plan.take_error() != 0
    assert plan.take_error() == 0  # reset by reading
    assert bool((buf[nb:] == 0x5A).all())
    one = torch.full((cs,), 0x5A, dtype=torch.uint8, device="cuda")
    plan.decode_ctx(di[1:], one, P)
    torch.cuda.synchronize()
    assert plan.take_error() == 0
    assert torch.equal(buf[cs:2 * cs], one)


def test_plan_argument_checks():
    """The Python wrapper refuses tensors the C-ABI would mis-address."""
    torch = _torch()
    import quadiron_amd as qa
    plan = qa.Plan(16, 48)
    good = torch.zeros((2, 16, 256), dtype=torch.int16, device="cuda")
    out = torch.zeros((2, 64, 256), dtype=torch.int16, device="cuda")
    with pytest.raises(TypeError):
        plan.encode(good.float(), out)
    with pytest.raises(TypeError):
        plan.encode(good.cpu(), out)
    with pytest.raises(ValueError):
        plan.encode(good[:, :8], out)
    with pytest.raises(ValueError):
        plan.encode(good.transpose(1, 2).contiguous().transpose(1, 2), out)
    with pytest.raises(ValueError):
        plan.encode(good, out[:, :32])
    cnt = torch.zeros(2 * 64, dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        plan.encode(good, out, cnt, torch.zeros(10, dtype=torch.int32,
                                                device="cuda"), 64)


# ------------------------------------------------------------------- RS-NF4

def _nf4_roundtrip(ws, k, m, data, cap, missing):
    import quadiron_amd as qa
    f = qa.Nf4(ws, k, m)
    no = f.n_outputs
    B = data.shape[1]
    outs = np.zeros((no, B), np.uint8)
    oor = np.zeros((no, cap), np.uint32)
    flags = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    f.encode([np.ascontiguousarray(data[i]) for i in range(k)],
             [outs[i] for i in range(no)], oor, flags, cnt)
    decs = []
    for miss in missing:
        dec = [np.zeros(B, np.uint8) for _ in range(k)]
        par = [None if miss[i] else outs[i].copy() for i in range(no)]
        assert f.decode(dec, par, oor, flags, cnt,
                        np.ascontiguousarray(miss, np.int32),
                        np.ones(k, np.int32)) == 1
        decs.append(np.stack(dec))
    return outs, oor, flags, cnt, decs


@pytest.mark.parametrize("name", golden_names("nf4_"))
def test_nf4_vs_reference_golden(hip_lib, name):
    """RS-NF4 through qi_nf4_* (qi::fec::RsNf4 on the RS-FNT device path)
    against RsNf4<T> outputs, including multi-component OOR words and a
    partial trailing word."""
    g = load(name)
    ws, k, m, pkt, B, cap = (int(v) for v in g["params"])
    outs, oor, flags, cnt, decs = _nf4_roundtrip(ws, k, m, g["data"], cap,
                                                 g["missing"])
    assert (outs == g["outputs"]).all()
    assert (cnt == g["oor_count"]).all()
    assert (oor == g["oor"]).all() and (flags == g["flags"]).all()
    for p, dec in enumerate(decs):
        assert (dec == g["decoded"][p]).all()


def test_nf4_vs_oracle_large(hip_lib):
    """A larger random RS-NF4 block (word_size 8, k=16, m=48) against the
    oracle, bit-exact (parity unpinned beyond the fixtures' sizes; the
    oracle itself is pinned by test_oracle_nf4_vs_reference)."""
    from qi_testlib import oracle_nf4_encode_blocks, oracle_nf4_decode_blocks
    rng = np.random.default_rng(41)
    ws, k, m, B = 8, 16, 48, 3 * 65536 + 8
    data = rng.integers(0, 256, (k, B), dtype=np.uint8)
    cap = 64 + B // 512
    miss = np.zeros(k + m, np.int32)
    miss[rng.choice(k + m, m, replace=False)] = 1
    outs, oor, flags, cnt, decs = _nf4_roundtrip(ws, k, m, data, cap, [miss])
    o_outs, o_oor, o_flags, o_cnt = oracle_nf4_encode_blocks(ws, k, m, data,
                                                             cap)
    assert (outs == o_outs).all() and (cnt == o_cnt).all()
    assert (oor == o_oor).all() and (flags == o_flags).all()
    ok, o_dec = oracle_nf4_decode_blocks(ws, k, m, o_outs, o_oor, o_flags,
                                         o_cnt, miss)
    assert ok == 1 and (decs[0] == o_dec).all()
    assert (decs[0] == data).all()


def test_nf4_bad_word_size(hip_lib):
    assert hip_lib.qi_nf4_new(3, 4, 4) is None
    assert hip_lib.qi_nf4_new(16, 4, 4) is None


# -------------------------------------------- stream API (pinned pipeline)

@pytest.mark.parametrize("k,m,sys_,B", [
    (4, 4, 0, 20 * 2**20 + 6),    # 3 chunks of 8 MiB, ragged tail
    (16, 48, 0, 3 * 2**20 + 2),   # one partial chunk
    (10, 6, 1, 9 * 2**20 + 1001), # systematic, 2 chunks, odd byte count
])
def test_streams_match_blocks(hip_lib, k, m, sys_, B):
    """encode/decode_streams_vertical (two-slot pinned pipeline over chunks)
    give the block API's and the oracle's outputs and OOR marks, and decode
    to the oracle's decode of the same fragments (== the data) -- including
    crafted OOR columns in every chunk."""
    import quadiron_amd as qa
    rng = np.random.default_rng(B)
    data = rng.integers(0, 256, (k, B), dtype=np.uint8)
    words = B // 2
    lanes = np.ascontiguousarray(data[:, :2 * words]).view(np.uint16)
    for c0 in range(0, words, 4 * 2**20):
        _craft(k, m, sys_, lanes, rng, 4, col_range=(c0, min(words, c0 + 4096)))
    data[:, :2 * words] = lanes.view(np.uint8)
    f = qa.Fec(k, m, sys_)
    no = f.n_outputs
    cap = 512
    outs_b, oor_b, cnt_b = fec_encode(hip_lib, k, m, sys_, data, cap)
    assert cnt_b.sum() > 0
    outs = np.zeros((no, B), np.uint8)
    oor = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    rows = [np.ascontiguousarray(data[i]) for i in range(k)]
    assert hip_lib.qi_fec_encode_streams(
        f.h, qa.ptr_array(rows), B, qa.ptr_array([outs[i] for i in range(no)]),
        oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
        cap) == 0
    # the block API codes whole words only (block_size = bytes / word_size,
    # src/fec_base.h:1083) while a stream's last packet keeps its partial
    # word (zero padded, read_bytes written, src/fec_base.h:504-538)
    assert (outs[:, :2 * words] == outs_b[:, :2 * words]).all()
    assert (cnt == cnt_b).all() and (oor == oor_b).all()
    miss = np.zeros(k + m, np.int32)
    miss[rng.choice(k + m, m, replace=False)] = 1
    din = ([None if miss[i] else rows[i] for i in range(k)] if sys_ else None)
    par = [None if miss[(k + i) if sys_ else i] else outs[i] for i in range(no)]
    dec = [np.zeros(B, np.uint8) for _ in range(k)]
    rc = hip_lib.qi_fec_decode_streams(
        f.h, qa.ptr_array(din) if din is not None else None, qa.ptr_array(par),
        B, oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p), cap,
        qa.ptr_array(dec))
    assert rc == 1
    if sys_ and not miss[:k].any():
        check_windows_vs_oracle(k, m, sys_, data, outs, oor, cnt,
                                chunk_windows(words))
        return  # data in clear: nothing decoded (src/fec_base.h:931-932)
    # an odd-sized stream's last coded word lost its high byte when written
    # (read_bytes), so only whole words decode back -- as in the reference
    assert (np.stack(dec)[:, :2 * words] == data[:, :2 * words]).all()
    # and against the oracle, not only the block API: outputs, OOR lists and
    # the decode, window by window (start, every chunk seam -- where the
    # crafted OOR columns sit -- and the tail)
    check_windows_vs_oracle(k, m, sys_, data, outs, oor, cnt,
                            chunk_windows(words), miss, np.stack(dec))
