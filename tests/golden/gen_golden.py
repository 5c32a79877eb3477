#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference and `make -C oracle ref`):

    python tests/golden/gen_golden.py

The expected outputs are produced by oracle/_ref/libqiref.so, i.e. QuadIron's
own RsFnt<uint32_t> (FecCode::encode_blocks_vertical / decode_blocks_vertical,
src/fec_base.h:1066-1321) and Properties::fnt_serialize/deserialize
(src/property.h:104-142) compiled from the reference sources.  The only input
the plain-C oracle contributes is the *crafting* of OOR-forcing data columns
(choose d0 so that a chosen output equals 65536); the expected values for
those columns still come from the reference.

Fixtures are .npz files holding only integer arrays (load with
numpy.load(allow_pickle=False)).
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "libqiref.so")
ORA = os.path.join(ROOT, "oracle", "liboracle.so")
Q = 65537


class Codec(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ["sys", "k", "m", "code_len", "n_outputs", "n", "data_len",
                 "len_2k"]] + [("r", C.c_uint32)]


def ptrs(arrs):
    p = (C.POINTER(C.c_uint8) * len(arrs))()
    for i, a in enumerate(arrs):
        p[i] = a.ctypes.data_as(C.POINTER(C.c_uint8)) if a is not None else None
    return p


def vp(a):
    return a.ctypes.data_as(C.c_void_p)


def craft_oor(ora, codec, data, rng, n_cols):
    """Overwrite data[0] at n_cols random columns so that one chosen output
    row equals 65536 there (exercises the OOR side channel)."""
    k, no = codec.k, codec.n_outputs
    words = data.shape[1] // 2
    first = k if codec.sys else 0
    cw = (C.c_uint32 * codec.n)()
    din = (C.c_uint32 * k)()
    ids = (C.c_uint32 * k)(*range(k))
    ctx = C.create_string_buffer(4 + 16 * 4096 + 64)
    if codec.sys:
        ora.qo_ctx_init(C.byref(codec), ctx, ids)

    def enc(vals):
        for t in range(k):
            din[t] = int(vals[t])
        ora.qo_encode_column(C.byref(codec), ctx if codec.sys else None,
                             din, cw)
        return [cw[first + i] for i in range(no)]

    e0 = [1] + [0] * (k - 1)
    a = enc(e0)
    done = 0
    for j in rng.permutation(words):
        if done >= n_cols:
            break
        col = data[:, 2 * j].astype(np.uint32) | (
            data[:, 2 * j + 1].astype(np.uint32) << 8)
        col[0] = 0
        b = enc(col)
        i = int(rng.integers(0, no))
        if a[i] == 0:
            continue
        d0 = ((65536 - b[i]) % Q) * pow(a[i], Q - 2, Q) % Q
        if d0 == 65536:
            continue
        data[0, 2 * j] = d0 & 0xFF
        data[0, 2 * j + 1] = d0 >> 8
        done += 1


def _gen_blocks(ref, ora, name, k, m, sys_, pkt, block_bytes, seed,
               n_patterns, n_craft, out_dir):
    rng = np.random.default_rng(seed)
    codec = Codec()
    assert ora.qo_codec_init(C.byref(codec), k, m, sys_) == 0
    no = codec.n_outputs
    data = rng.integers(0, 256, (k, block_bytes), dtype=np.uint8)
    if n_craft:
        craft_oor(ora, codec, data, rng, n_craft)
    cap = 64 + block_bytes // 2048
    outs = np.zeros((no, block_bytes), np.uint8)
    oor = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    rows = [data[i].copy() for i in range(k)]
    orow = [outs[i] for i in range(no)]
    ref.ref_encode_blocks(sys_, k, m, C.c_size_t(pkt), ptrs(rows), ptrs(orow),
                          C.c_size_t(block_bytes), vp(oor), vp(cnt),
                          C.c_uint32(cap))
    assert (cnt <= cap).all()
    missing = np.zeros((n_patterns, k + m), np.int32)
    decoded = np.zeros((n_patterns, k, block_bytes), np.uint8)
    for p in range(n_patterns):
        miss = rng.choice(k + m, m, replace=False)
        missing[p, miss] = 1
        dec = [np.zeros(block_bytes, np.uint8) if (not sys_ or missing[p, i])
               else data[i].copy() for i in range(k)]
        par = [None if missing[p, (k + i) if sys_ else i] else outs[i].copy()
               for i in range(no)]
        wanted = np.ones(k, np.int32)
        ok = ref.ref_decode_blocks(sys_, k, m, C.c_size_t(pkt), ptrs(dec),
                                   ptrs(par), vp(oor), vp(cnt),
                                   C.c_uint32(cap), vp(missing[p]),
                                   vp(wanted), C.c_size_t(block_bytes))
        assert ok == 1
        decoded[p] = np.stack(dec)
    np.savez_compressed(
        os.path.join(out_dir, name + ".npz"),
        params=np.array([k, m, sys_, pkt, block_bytes, cap], np.int64),
        data=data, outputs=outs, oor=oor, oor_count=cnt, missing=missing,
        decoded=decoded)
    print(f"{name}: k={k} m={m} sys={sys_} block={block_bytes} "
          f"oor={int(cnt.sum())}")


def _gen_cabi(ref, ora, name, k, m, sys_, block_bytes, seed, n_patterns,
             n_craft, out_dir):
    """C-ABI fixtures: full fragment buffers (FNT1 header + payload)."""
    rng = np.random.default_rng(seed)
    codec = Codec()
    assert ora.qo_codec_init(C.byref(codec), k, m, sys_) == 0
    md = ref.ref_metadata_size(C.c_size_t(block_bytes))
    payload = rng.integers(0, 256, (k, block_bytes), dtype=np.uint8)
    if n_craft:
        craft_oor(ora, codec, payload, rng, n_craft)
    data = np.zeros((k, md + block_bytes), np.uint8)
    data[:, md:] = payload
    par = np.zeros((m, md + block_bytes), np.uint8)
    no = codec.n_outputs
    wanted = np.ones(no, np.int32)
    d = [data[i].copy() for i in range(k)]
    p = [par[i].copy() for i in range(m)]
    rc = ref.ref_c_encode(sys_, k, m, ptrs(d), ptrs(p), vp(wanted),
                          C.c_size_t(block_bytes))
    assert rc == 0
    enc_data, enc_par = np.stack(d), np.stack(p)
    missing = np.zeros((n_patterns, k + m), np.int32)
    dec = np.zeros((n_patterns, k, md + block_bytes), np.uint8)
    dest = np.zeros(n_patterns, np.int32)
    rec = np.zeros((n_patterns, md + block_bytes), np.uint8)
    for t in range(n_patterns):
        miss = rng.choice(k + m, m, replace=False)
        missing[t, miss] = 1
        D = [enc_data[i].copy() if not missing[t, i]
             else np.zeros(md + block_bytes, np.uint8) for i in range(k)]
        P = [enc_par[i].copy() if not missing[t, k + i]
             else np.zeros(md + block_bytes, np.uint8) for i in range(m)]
        assert ref.ref_c_decode(sys_, k, m, ptrs(D), ptrs(P),
                                vp(missing[t]), C.c_size_t(block_bytes)) == 0
        dec[t] = np.stack(D)
        dest[t] = int(rng.choice(miss))
        D = [enc_data[i].copy() if not missing[t, i]
             else np.zeros(md + block_bytes, np.uint8) for i in range(k)]
        P = [enc_par[i].copy() if not missing[t, k + i]
             else np.zeros(md + block_bytes, np.uint8) for i in range(m)]
        assert ref.ref_c_reconstruct(sys_, k, m, ptrs(D), ptrs(P),
                                     vp(missing[t]), C.c_uint(dest[t]),
                                     C.c_size_t(block_bytes)) == 0
        rec[t] = (D + P)[dest[t]]
    np.savez_compressed(
        os.path.join(out_dir, name + ".npz"),
        params=np.array([k, m, sys_, block_bytes, md], np.int64),
        data=data, enc_data=enc_data, enc_parity=enc_par, missing=missing,
        decoded=dec, dest=dest, reconstructed=rec)
    print(f"{name}: C-ABI k={k} m={m} sys={sys_} block={block_bytes} md={md}")


def all_patterns(k, m):
    """Every decodable erasure set of a (k, m) code, 0 .. m missing, in the
    order of test/quadiron_c_utest.cpp:58-74,283-295 (combinations of
    size i = 0..m, lexicographic, from prev_permutation over a selector with
    the first i entries set)."""
    import itertools
    return [list(c) for i in range(m + 1)
            for c in itertools.combinations(range(k + m), i)]


def _gen_cabi_scn(ref, ora, name, k, m, sys_, block_bytes, seed, patterns,
                  n_craft, out_dir):
    """C-ABI scenario fixtures: the reference's own C-ABI test sequence,
    test_encode_decode_reconstruct (test/quadiron_c_utest.cpp:109-281), run
    through oracle/_ref for every given erasure pattern:

      encode (all outputs wanted) -> zero the missing fragments -> decode ->
      (non-sys: put the k coded fragments back) -> zero the missing fragments
      -> reconstruct every missing data index, then every missing parity
      index, in ascending order, on the SAME buffers (so later reconstructs
      see the earlier ones' results in buffers still flagged missing).

    Stored: the encoded fragments; per pattern the decoded fragments' FNT1
    headers, and per reconstruct (rec_pat / rec_dest) the reconstructed
    fragment's FNT1 header.  Payloads are not stored twice: the reference's
    outputs are asserted here to be the input data (decode; systematic data
    reconstruct) or the encoded fragment, header included (every other
    reconstruct), exactly the reference test's own checks."""
    rng = np.random.default_rng(seed)
    codec = Codec()
    assert ora.qo_codec_init(C.byref(codec), k, m, sys_) == 0
    md = ref.ref_metadata_size(C.c_size_t(block_bytes))
    L = md + block_bytes
    payload = rng.integers(0, 256, (k, block_bytes), dtype=np.uint8)
    if n_craft:
        craft_oor(ora, codec, payload, rng, n_craft)
    data = np.zeros((k, L), np.uint8)
    data[:, md:] = payload
    d = [data[i].copy() for i in range(k)]
    p = [np.zeros(L, np.uint8) for _ in range(m)]
    wanted = np.ones(codec.n_outputs, np.int32)
    assert ref.ref_c_encode(sys_, k, m, ptrs(d), ptrs(p), vp(wanted),
                            C.c_size_t(block_bytes)) == 0
    enc_data, enc_par = np.stack(d), np.stack(p)
    missing = np.zeros((len(patterns), k + m), np.int32)
    dec_hdr = np.zeros((len(patterns), k, md), np.uint8)
    rec_pat, rec_dest, rec_hdr = [], [], []
    for t, miss in enumerate(patterns):
        missing[t, miss] = 1
        mv = missing[t]
        D = [enc_data[i].copy() for i in range(k)]
        P = [enc_par[i].copy() for i in range(m)]
        for i in miss:
            (D + P)[i][:] = 0
        assert ref.ref_c_decode(sys_, k, m, ptrs(D), ptrs(P), vp(mv),
                                C.c_size_t(block_bytes)) == 0
        for i in range(k):
            assert (D[i][md:] == payload[i]).all(), (name, miss, i)
            dec_hdr[t, i] = D[i][:md]
        if not sys_:
            D = [enc_data[i].copy() for i in range(k)]
        for i in miss:
            (D + P)[i][:] = 0
        for dest in sorted(miss):
            assert ref.ref_c_reconstruct(sys_, k, m, ptrs(D), ptrs(P), vp(mv),
                                         C.c_uint(dest),
                                         C.c_size_t(block_bytes)) == 0
            got = (D + P)[dest]
            # the reference test's own checks (quadiron_c_utest.cpp:241-276)
            if dest < k and sys_:
                assert (got[md:] == payload[dest]).all()
            else:
                exp = (enc_par[dest - k] if dest >= k
                       else enc_data[dest])
                assert (got == exp).all(), (name, miss, dest)
            rec_pat.append(t)
            rec_dest.append(dest)
            rec_hdr.append(got[:md].copy())
    rec_hdr = np.stack(rec_hdr) if rec_hdr else np.zeros((0, md), np.uint8)
    np.savez_compressed(
        os.path.join(out_dir, name + ".npz"),
        params=np.array([k, m, sys_, block_bytes, md], np.int64),
        data=data, enc_data=enc_data, enc_parity=enc_par, missing=missing,
        decoded_hdr=dec_hdr, rec_pat=np.array(rec_pat, np.int32),
        rec_dest=np.array(rec_dest, np.int32), rec_hdr=rec_hdr)
    print(f"{name}: C-ABI scenarios k={k} m={m} sys={sys_} "
          f"block={block_bytes} patterns={len(patterns)} "
          f"reconstructs={len(rec_dest)}")


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    ref = C.CDLL(REF)
    ora = C.CDLL(ORA)
    ora.qo_nth_root.restype = C.c_uint32
    out = HERE
    # `python gen_golden.py name ...` regenerates only the named fixtures
    only = set(sys.argv[1:])

    def gen_blocks(*a):
        if not only or a[2] in only:
            _gen_blocks(*a)

    def gen_cabi(*a):
        if not only or a[2] in only:
            _gen_cabi(*a)
    # block-level (vertical) fixtures; pkt sizes differ on purpose (outputs
    # are pkt-size invariant)
    gen_blocks(ref, ora, "blk_k4_m4", 4, 4, 0, 512, 4096 + 6, 11, 6, 8, out)
    gen_blocks(ref, ora, "blk_k16_m48", 16, 48, 0, 1024, 8192 + 2, 12, 6, 24,
               out)
    gen_blocks(ref, ora, "blk_k16_m48_sys", 16, 48, 1, 1024, 8192, 13, 6, 24,
               out)
    gen_blocks(ref, ora, "blk_k64_m960", 64, 960, 0, 2048, 512, 14, 3, 12, out)
    gen_blocks(ref, ora, "blk_k3_m3_sys", 3, 3, 1, 8, 2000, 15, 6, 6, out)
    gen_blocks(ref, ora, "blk_k9_m5", 9, 5, 0, 8, 2001, 16, 6, 6, out)
    gen_blocks(ref, ora, "blk_k10_m6_sys", 10, 6, 1, 1024, 4096, 17, 6, 8, out)
    # C-ABI fixtures (pkt_size 1024 inside, headers in front)
    gen_cabi(ref, ora, "cabi_k3_m3", 3, 3, 0, 10000, 21, 6, 4, out)
    gen_cabi(ref, ora, "cabi_k3_m3_sys", 3, 3, 1, 10000, 22, 6, 4, out)
    gen_cabi(ref, ora, "cabi_k16_m48", 16, 48, 0, 4096 + 2, 23, 3, 24, out)
    gen_cabi(ref, ora, "cabi_k4_m4_big", 4, 4, 0, 2 * 65536 + 10, 25, 2, 12,
             out)
    gen_cabi(ref, ora, "cabi_k8_m4_sys", 8, 4, 1, 3 * 4096 + 2, 24, 6, 8, out)
    # k > 64: the NTT-structured general path (round 2)
    gen_blocks(ref, ora, "blk_k200_m56", 200, 56, 0, 1024, 1500 + 2, 31, 3, 12,
               out)
    gen_blocks(ref, ora, "blk_k200_m56_sys", 200, 56, 1, 512, 1500, 32, 3, 12,
               out)
    gen_blocks(ref, ora, "blk_k256_m768", 256, 768, 0, 256, 800, 33, 2, 12, out)
    gen_blocks(ref, ora, "blk_k100_m28", 100, 28, 0, 64, 1200 + 6, 34, 3, 8, out)
    gen_cabi(ref, ora, "cabi_k200_m56", 200, 56, 0, 1500 + 2, 35, 2, 8, out)
    gen_cabi(ref, ora, "cabi_k130_m30_sys", 130, 30, 1, 2000, 36, 2, 8, out)
    # k > 256: the NTT-structured path (k <= 256 moved to the matrix cores)
    gen_blocks(ref, ora, "blk_k300_m212", 300, 212, 0, 128, 600 + 2, 37, 2, 8, out)
    gen_blocks(ref, ora, "blk_k260_m30_sys", 260, 30, 1, 256, 512, 38, 2, 8, out)
    # max(n, len_2k) > 2048: the multi-pass NTT engine (ntt_pass_kernel over
    # HBM scratch) -- n = 4096 non-systematic and systematic, len_2k = 4096
    # > n = 2048, and n = 16384 (round 3)
    gen_blocks(ref, ora, "blk_k300_m3796", 300, 3796, 0, 64, 256 + 2, 39, 2, 8, out)
    gen_blocks(ref, ora, "blk_k260_m3000_sys", 260, 3000, 1, 128, 256, 40, 2, 8, out)
    gen_blocks(ref, ora, "blk_k1100_m100", 1100, 100, 0, 64, 256 + 6, 41, 2, 8, out)
    gen_blocks(ref, ora, "blk_k300_m16000", 300, 16000, 0, 32, 64 + 2, 42, 1, 8, out)
    # 256 < k <= 384 at whole 1024-word tiles: the matrix cores at KS = 20 /
    # 24 (round 3; ragged widths of these codes stay on the NTT engine)
    gen_blocks(ref, ora, "blk_k300_m212_w1024", 300, 212, 0, 256, 2048, 43, 2, 8, out)
    gen_blocks(ref, ora, "blk_k384_m128_sys_w1024", 384, 128, 1, 512, 2048, 44, 2, 8,
               out)
    # few erasures (n - k <= 64): the erasure decode of the NTT engine (round
    # 4) -- n = 1024 and 512, systematic, and n = 2048 (len_2k = 4096: the
    # encode on the multi-pass engine)
    gen_blocks(ref, ora, "blk_k1000_m24", 1000, 24, 0, 64, 256 + 6, 45, 2, 8, out)
    gen_blocks(ref, ora, "blk_k500_m12_sys", 500, 12, 1, 128, 512, 46, 2, 8, out)
    gen_blocks(ref, ora, "blk_k2000_m48", 2000, 48, 0, 32, 128 + 2, 47, 2, 8, out)

    # 384 < k <= 640 at a whole 1024-word tile: the decode on the matrix
    # cores at KS = 40 in two K chunks (round 6)
    gen_blocks(ref, ora, "blk_k400_m100_w1024", 400, 100, 0, 256, 2048, 55, 1, 10, out)
    # systematic 384 < k <= 640 (round 6): the encode from the closed-form
    # Lagrange generator and the two-region decode, both at KS = 40
    gen_blocks(ref, ora, "blk_k450_m200_sys_w1024", 450, 200, 1, 256, 2048, 56, 1, 10, out)

    def gen_scn(*a):
        if not only or a[2] in only:
            _gen_cabi_scn(*a)
    # the reference's exhaustive C-ABI scenario test (round 6):
    # test/quadiron_c_utest.cpp:283-309 -- (3, 3), block 10000, every
    # 0..m-erasure pattern (42 per type), every missing index reconstructed
    gen_scn(ref, ora, "cabiscn_k3_m3", 3, 3, 0, 10000, 51,
            all_patterns(3, 3), 4, out)
    gen_scn(ref, ora, "cabiscn_k3_m3_sys", 3, 3, 1, 10000, 52,
            all_patterns(3, 3), 4, out)
    # cfg2-shaped (16, 48) at a 64 KiB + 2 block: fewer-than-m erasures, so
    # the decoder's first-k choice (src/fec_base.h:1199-1236) is exercised,
    # with data and parity fragments missing together
    cfg2_pats = [[], [3], [0, 17, 40], [1, 2, 5, 15, 16, 33, 63],
                 list(range(0, 32, 2)) + [47, 50],
                 [i for i in range(64) if i % 4 != 1][:47]]
    gen_scn(ref, ora, "cabiscn_k16_m48", 16, 48, 0, 65536 + 2, 53,
            cfg2_pats, 24, out)


if __name__ == "__main__":
    main()
