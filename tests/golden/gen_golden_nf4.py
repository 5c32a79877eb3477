#!/usr/bin/env python3
"""Generate the RS-NF4 golden fixtures (tests/golden/nf4_*.npz) from the
REFERENCE itself: RsNf4<T>(word_size, k, m, pkt) (src/fec_rs_nf4.h) through
FecCode::encode_blocks_vertical / decode_blocks_vertical, compiled from the
reference sources into oracle/_ref/libqiref.so (oracle/ref_driver.cpp
ref_nf4_*).  Run in the build container:

    make -C oracle ref && python tests/golden/gen_golden_nf4.py

OOR marks are (word offset, component mask) pairs.  block_bytes need not be
a multiple of word_size: the trailing bytes of a partial word are left
untouched (block_size = block_size_bytes / word_size, src/fec_base.h:1083).
The only input the plain-C oracle contributes is the crafting of OOR-forcing
16-bit lanes (gen_golden.craft_oor); expected values come from the reference.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gen_golden import ORA, REF, Codec, craft_oor, ptrs, vp  # noqa: E402


def craft_word(ora, codec, data, word, g, row):
    """Make every component of `word` equal 65536 on output `row` (a
    multi-component OOR mark) by choosing data[0] at each of its lanes."""
    k, Q = codec.k, 65537
    cw = (C.c_uint32 * codec.n)()
    din = (C.c_uint32 * k)()

    def enc(vals):
        for t in range(k):
            din[t] = int(vals[t])
        ora.qo_encode_column(C.byref(codec), None, din, cw)
        return cw[row]

    a = enc([1] + [0] * (k - 1))
    assert a != 0
    for comp in range(g):
        lane = word * g + comp
        col = data[:, 2 * lane].astype(np.uint32) | (
            data[:, 2 * lane + 1].astype(np.uint32) << 8)
        col[0] = 0
        d0 = ((65536 - enc(col)) % Q) * pow(a, Q - 2, Q) % Q
        if d0 == 65536:
            continue  # not reachable with a u16 data symbol
        data[0, 2 * lane] = d0 & 0xFF
        data[0, 2 * lane + 1] = d0 >> 8


def gen_nf4(ref, ora, name, ws, k, m, pkt, block_bytes, seed, n_patterns,
            n_craft, out_dir):
    rng = np.random.default_rng(seed)
    codec = Codec()
    assert ora.qo_codec_init(C.byref(codec), k, m, 0) == 0
    no = ref.ref_nf4_n_outputs(ws, k, m)
    assert no == codec.n_outputs
    data = rng.integers(0, 256, (k, block_bytes), dtype=np.uint8)
    if n_craft:
        # every 16-bit lane is an RS-FNT column: craft them like RS-FNT's
        craft_oor(ora, codec, data, rng, n_craft)
        g = ws // 2
        for word in rng.choice(block_bytes // ws, 4, replace=False):
            craft_word(ora, codec, data, int(word), g,
                       int(rng.integers(1, k + m)))
    cap = 64 + block_bytes // 1024
    outs = np.zeros((no, block_bytes), np.uint8)
    oor = np.zeros((no, cap), np.uint32)
    flags = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    rows = [data[i].copy() for i in range(k)]
    ref.ref_nf4_encode_blocks(ws, k, m, C.c_size_t(pkt), ptrs(rows),
                              ptrs([outs[i] for i in range(no)]),
                              C.c_size_t(block_bytes), vp(oor), vp(flags),
                              vp(cnt), C.c_uint32(cap))
    assert (cnt <= cap).all()
    missing = np.zeros((n_patterns, k + m), np.int32)
    decoded = np.zeros((n_patterns, k, block_bytes), np.uint8)
    for p in range(n_patterns):
        missing[p, rng.choice(k + m, m, replace=False)] = 1
        dec = [np.zeros(block_bytes, np.uint8) for _ in range(k)]
        par = [None if missing[p, i] else outs[i].copy() for i in range(no)]
        wanted = np.ones(k, np.int32)
        assert ref.ref_nf4_decode_blocks(
            ws, k, m, C.c_size_t(pkt), ptrs(dec), ptrs(par), vp(oor),
            vp(flags), vp(cnt), C.c_uint32(cap), vp(missing[p]), vp(wanted),
            C.c_size_t(block_bytes)) == 1
        decoded[p] = np.stack(dec)
    np.savez_compressed(
        os.path.join(out_dir, name + ".npz"),
        params=np.array([ws, k, m, pkt, block_bytes, cap], np.int64),
        data=data, outputs=outs, oor=oor, flags=flags, oor_count=cnt,
        missing=missing, decoded=decoded)
    multi = int(sum(bin(int(f)).count("1") > 1
                    for i in range(no) for f in flags[i, :cnt[i]]))
    print(f"{name}: NF4 w={ws} k={k} m={m} block={block_bytes} "
          f"marks={int(cnt.sum())} multi-component={multi}")


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    ref = C.CDLL(REF)
    ora = C.CDLL(ORA)
    gen_nf4(ref, ora, "nf4_w2_k4_m4", 2, 4, 4, 64, 2048 + 2, 31, 4, 6, HERE)
    gen_nf4(ref, ora, "nf4_w4_k16_m48", 4, 16, 48, 256, 8192 + 6, 32, 4, 48,
            HERE)
    gen_nf4(ref, ora, "nf4_w8_k10_m6", 8, 10, 6, 128, 4096 + 4, 33, 4, 16,
            HERE)
    gen_nf4(ref, ora, "nf4_w8_k16_m48", 8, 16, 48, 512, 8192, 34, 3, 64, HERE)


if __name__ == "__main__":
    main()
