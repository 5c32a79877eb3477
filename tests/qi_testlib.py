"""Shared test helpers: ctypes access to the CPU oracle (test infrastructure)
and golden-fixture loading.  Product code never imports this module."""
import ctypes as C
import glob
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
Q = 65537


class Codec(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ["sys", "k", "m", "code_len", "n_outputs", "n", "data_len",
                 "len_2k"]] + [("r", C.c_uint32)]


_oracle = None


def oracle():
    """Load (building if needed) the plain-C oracle."""
    global _oracle
    if _oracle is None:
        src = os.path.join(ROOT, "oracle", "qi_oracle.c")
        if (not os.path.exists(ORACLE_SO)
                or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src)):
            subprocess.check_call(["make", "-s", "-C",
                                   os.path.join(ROOT, "oracle")])
        lib = C.CDLL(ORACLE_SO)
        for fn in ("qo_add", "qo_sub", "qo_mul", "qo_exp", "qo_inv",
                   "qo_nth_root", "qo_code_len"):
            getattr(lib, fn).restype = C.c_uint32
        _oracle = lib
    return _oracle


def ptrs(arrs):
    p = (C.POINTER(C.c_uint8) * len(arrs))()
    for i, a in enumerate(arrs):
        p[i] = (a.ctypes.data_as(C.POINTER(C.c_uint8))
                if a is not None else None)
    return p


def vp(a):
    return a.ctypes.data_as(C.c_void_p)


def codec(k, m, sys_):
    c = Codec()
    assert oracle().qo_codec_init(C.byref(c), k, m, int(sys_)) == 0
    return c


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"),
                        allow_pickle=False))


def golden_names(prefix):
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def check_cabi_scenarios(g, encode, decode, reconstruct):
    """Replay a `cabiscn_*` fixture (tests/golden/gen_golden.py
    `_gen_cabi_scn`): the reference's C-ABI test sequence
    (test/quadiron_c_utest.cpp:109-281) for every stored erasure pattern,
    through the given encode(D, P, wanted, B) / decode(D, P, miss, B) /
    reconstruct(D, P, miss, dest, B) callables (the product's
    quadiron_fnt32_* or the oracle's qo_fnt32_*), on the same mutated
    buffers, comparing every fragment byte for byte: FNT1 headers against
    the reference's, payloads against the data / encoded fragments the
    reference produced."""
    k, m, sys_, B, md = (int(v) for v in g["params"])
    L = md + B
    payload = g["data"][:, md:]
    d = [g["data"][i].copy() for i in range(k)]
    p = [np.zeros(L, np.uint8) for _ in range(m)]
    wanted = np.ones(m if sys_ else k + m, np.int32)
    assert encode(d, p, wanted, B) == 0
    assert (np.stack(d) == g["enc_data"]).all()
    assert (np.stack(p) == g["enc_parity"]).all()
    enc = list(g["enc_data"]) + list(g["enc_parity"])
    r = 0
    for t in range(len(g["missing"])):
        miss = np.ascontiguousarray(g["missing"][t], np.int32)
        gone = np.flatnonzero(miss).tolist()
        D = [g["enc_data"][i].copy() for i in range(k)]
        P = [g["enc_parity"][i].copy() for i in range(m)]
        for i in gone:
            (D + P)[i][:] = 0
        assert decode(D, P, miss, B) == 0, gone
        for i in range(k):
            assert (D[i][:md] == g["decoded_hdr"][t, i]).all(), (gone, i)
            assert (D[i][md:] == payload[i]).all(), (gone, i)
        if not sys_:
            D = [g["enc_data"][i].copy() for i in range(k)]
        for i in gone:
            (D + P)[i][:] = 0
        for dest in sorted(gone):
            assert (g["rec_pat"][r], g["rec_dest"][r]) == (t, dest)
            assert reconstruct(D, P, miss, dest, B) == 0, (gone, dest)
            got = (D + P)[dest]
            assert (got[:md] == g["rec_hdr"][r]).all(), (gone, dest)
            exp = payload[dest] if (sys_ and dest < k) else enc[dest][md:]
            assert (got[md:] == exp).all(), (gone, dest)
            r += 1
    assert r == len(g["rec_dest"])


def oracle_encode_blocks(k, m, sys_, data, cap=None):
    """data: (k, B) uint8 -> outputs (n_outputs, B), oor (n_out, cap), cnt."""
    c = codec(k, m, sys_)
    B = data.shape[1]
    cap = cap or (64 + B // 2048)
    outs = np.zeros((c.n_outputs, B), np.uint8)
    oor = np.zeros((c.n_outputs, cap), np.uint32)
    cnt = np.zeros(c.n_outputs, np.uint32)
    rows = [np.ascontiguousarray(data[i]) for i in range(k)]
    oracle().qo_encode_blocks(C.byref(c), ptrs(rows),
                              ptrs([outs[i] for i in range(c.n_outputs)]),
                              C.c_size_t(B), vp(oor), vp(cnt),
                              C.c_uint32(cap))
    return outs, oor, cnt


def oracle_decode_blocks(k, m, sys_, outputs, oor, cnt, missing, data=None):
    """Decode from the encoded outputs with `missing` (code_len flags)."""
    c = codec(k, m, sys_)
    B = outputs.shape[1]
    dec = [np.zeros(B, np.uint8) if (not sys_ or missing[i] or data is None)
           else data[i].copy() for i in range(k)]
    par = [None if missing[(k + i) if sys_ else i] else outputs[i].copy()
           for i in range(c.n_outputs)]
    missing = np.ascontiguousarray(missing, np.int32)
    wanted = np.ones(k, np.int32)
    ok = oracle().qo_decode_blocks(C.byref(c), ptrs(dec), ptrs(par), vp(oor),
                                   vp(cnt), C.c_uint32(oor.shape[1]),
                                   vp(missing), vp(wanted), C.c_size_t(B))
    return ok, np.stack(dec)


def oracle_nf4_encode_blocks(ws, k, m, data, cap):
    """RS-NF4 (oracle): data (k, B) uint8 -> outputs, oor words, flags, cnt."""
    c = codec(k, m, 0)
    B = data.shape[1]
    outs = np.zeros((c.n_outputs, B), np.uint8)
    oor = np.zeros((c.n_outputs, cap), np.uint32)
    flags = np.zeros((c.n_outputs, cap), np.uint32)
    cnt = np.zeros(c.n_outputs, np.uint32)
    rows = [np.ascontiguousarray(data[i]) for i in range(k)]
    oracle().qo_nf4_encode_blocks(C.byref(c), ws, ptrs(rows),
                                  ptrs([outs[i] for i in range(c.n_outputs)]),
                                  C.c_size_t(B), vp(oor), vp(flags), vp(cnt),
                                  C.c_uint32(cap))
    return outs, oor, flags, cnt


def oracle_nf4_decode_blocks(ws, k, m, outputs, oor, flags, cnt, missing):
    c = codec(k, m, 0)
    B = outputs.shape[1]
    dec = [np.zeros(B, np.uint8) for _ in range(k)]
    par = [None if missing[i] else outputs[i].copy()
           for i in range(c.n_outputs)]
    missing = np.ascontiguousarray(missing, np.int32)
    wanted = np.ones(k, np.int32)
    ok = oracle().qo_nf4_decode_blocks(
        C.byref(c), ws, ptrs(dec), ptrs(par), vp(oor), vp(flags), vp(cnt),
        C.c_uint32(oor.shape[1]), vp(missing), vp(wanted), C.c_size_t(B))
    return ok, np.stack(dec)


def craft_oor_columns(k, m, sys_, data_rows, rng, n_cols, rows=None, col_range=None):
    """Force some outputs to 65536 (OOR) by solving for data row 0
    (optionally only on output `rows`, in columns `col_range`)."""
    o = oracle()
    c = codec(k, m, sys_)
    first = k if sys_ else 0
    cw = (C.c_uint32 * c.n)()
    din = (C.c_uint32 * k)()
    ctx = C.create_string_buffer(4 + 16 * 4096 + 64)
    if sys_:
        o.qo_ctx_init(C.byref(c), ctx, (C.c_uint32 * k)(*range(k)))

    def enc(vals):
        for t in range(k):
            din[t] = int(vals[t])
        o.qo_encode_column(C.byref(c), ctx if sys_ else None, din, cw)
        return [cw[first + i] for i in range(c.n_outputs)]

    a = enc([1] + [0] * (k - 1))
    P = data_rows.shape[1]
    lo, hi = col_range if col_range else (0, P)
    for j in lo + rng.choice(hi - lo, min(n_cols, hi - lo), replace=False):
        col = data_rows[:, j].astype(np.int64)
        col[0] = 0
        b = enc(col)
        i = int(rng.choice(rows)) if rows is not None else int(
            rng.integers(0, c.n_outputs))
        if a[i] == 0:
            continue
        d0 = ((65536 - b[i]) % Q) * pow(a[i], Q - 2, Q) % Q
        if d0 < 65536:
            data_rows[0, j] = d0


def _solve_mod(A, b):
    """x with A x = b (mod Q) by Gaussian elimination, or None if singular."""
    n = len(A)
    M = [list(A[i]) + [b[i]] for i in range(n)]
    for c in range(n):
        piv = next((r for r in range(c, n) if M[r][c] % Q), None)
        if piv is None:
            return None
        M[c], M[piv] = M[piv], M[c]
        inv = pow(M[c][c], Q - 2, Q)
        M[c] = [v * inv % Q for v in M[c]]
        for r in range(n):
            if r != c and M[r][c]:
                f = M[r][c]
                M[r] = [(vr - f * vc) % Q for vr, vc in zip(M[r], M[c])]
    return [M[i][n] for i in range(n)]


def craft_dense_oor(k, m, data_rows, rng, cols, rows, per_col):
    """Non-systematic: make `per_col` distinct outputs among `rows` equal
    65536 (OOR) in every column of `cols`, by solving for data rows
    0..per_col-1 of that column.  Returns the number of columns crafted."""
    o = oracle()
    c = codec(k, m, 0)
    cw = (C.c_uint32 * c.n)()
    din = (C.c_uint32 * k)()

    def enc(vals):
        for t in range(k):
            din[t] = int(vals[t])
        o.qo_encode_column(C.byref(c), None, din, cw)
        return [cw[i] for i in range(c.n_outputs)]

    G = [enc([1 if t == u else 0 for t in range(k)]) for u in range(per_col)]
    rows = list(rows)
    done = 0
    for j in cols:
        col = data_rows[:, j].astype(np.int64)
        col[:per_col] = 0
        b = enc(col)
        sel = rng.choice(rows, per_col, replace=False)
        A = [[G[u][int(i)] for u in range(per_col)] for i in sel]
        x = _solve_mod(A, [(65536 - b[int(i)]) % Q for i in sel])
        if x is None or any(v == 65536 for v in x):
            continue
        data_rows[:per_col, j] = x
        done += 1
    return done


def chunk_windows(words, chunk=1 << 21, width=4096):
    """Column windows [lo, hi) around the start, every stream-chunk boundary
    and the tail of a `words`-column block."""
    wins = {(0, min(words, width))}
    for c in range(chunk, words, chunk):
        wins.add((max(0, c - width // 2), min(words, c + width // 2)))
        wins.add((c, min(words, c + width)))
    wins.add((max(0, words - width), words))
    return sorted(wins)


def check_windows_vs_oracle(k, m, sys_, data, outs, oor, cnt, wins, missing=None,
                            dec=None):
    """The codes are column-independent, so a large block's outputs (and OOR
    marks, and decode) can be pinned to the oracle window by window: `data`
    (k, 2*words) bytes, `outs` the product's (n_outputs, >= 2*words) coded
    bytes with OOR lists oor/cnt (absolute word offsets)."""
    no = outs.shape[0]
    for lo, hi in wins:
        d = np.ascontiguousarray(data[:, 2 * lo:2 * hi])
        o_out, o_oor, o_cnt = oracle_encode_blocks(k, m, sys_, d, 64 + (hi - lo))
        assert (outs[:, 2 * lo:2 * hi] == o_out).all(), (lo, hi)
        for i in range(no):
            got = [int(w) - lo for w in oor[i, :cnt[i]] if lo <= w < hi]
            assert got == [int(w) for w in o_oor[i, :o_cnt[i]]], (lo, hi, i)
        if missing is not None:
            ok, o_dec = oracle_decode_blocks(k, m, sys_, o_out, o_oor, o_cnt,
                                             missing, d)
            assert ok == 1 and (dec[:, 2 * lo:2 * hi] == o_dec).all(), (lo, hi)
