#!/usr/bin/env python3
"""Host-inclusive RS-FNT rate (DESIGN.md "Host-inclusive rate").

The path starts and ends in host memory (shard files / socket buffers).  This
measures cfg2 (k=16, n=64, 64 KiB packets) with every byte crossing PCIe:

  encode:  pinned data rows --H2D--> encode --D2H--> pinned coded rows
  decode:  pinned received rows (k per stripe, packed in id order) --H2D-->
           decode_ctx_packed + decode_packed --D2H--> pinned data rows

in chunks of C stripes round-robin over 3 HIP streams (copy / compute
overlap), plus the raw pinned H2D / D2H copy rates.  Rates use the same
algorithmic bytes as bench.py: encode (k+n)*2P, decode 2k*2P per stripe.

    python tools/host_rate.py [--stripes 512] [--chunk 32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import quadiron_amd as qa  # noqa: E402
from bench import alg_bytes  # noqa: E402


def copy_rate(nbytes, h2d):
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    return 5 * nbytes / (time.perf_counter() - t) / 1e9


def cabi_rate(k, m, block):
    """The drop-in C-ABI (quadiron_fnt32_encode / _decode) on pageable numpy
    buffers of `block` payload bytes per fragment: what an unmodified caller
    of the reference API gets (synchronous per call)."""
    f = qa.QuadironFnt32(2, k, m, 0)
    md = f.metadata_size(block)
    rng = np.random.default_rng(3)
    data = [np.zeros(md + block, np.uint8) for _ in range(k)]
    par = [np.zeros(md + block, np.uint8) for _ in range(m)]
    orig = [rng.integers(0, 256, block, dtype=np.uint8) for _ in range(k)]
    wanted = np.ones(k + m, np.int32)
    t_enc = []
    for _ in range(2):
        for i in range(k):
            data[i][md:] = orig[i]
        t = time.perf_counter()
        assert f.encode(data, par, wanted, block) == 0
        t_enc.append(time.perf_counter() - t)
    coded = [d.copy() for d in data]
    missing = np.zeros(k + m, np.int32)
    missing[rng.choice(k + m, m, replace=False)] = 1
    t_dec = []
    for _ in range(2):
        for i in range(k):
            data[i][:] = coded[i]
        t = time.perf_counter()
        assert f.decode(data, par, missing, block) == 0
        t_dec.append(time.perf_counter() - t)
    ok = all((data[i][md:] == orig[i]).all() for i in range(k))
    n = 1
    while n < k + m:
        n *= 2
    P = block // 2
    enc_b, dec_b = alg_bytes(k, m, P)
    f.close()
    return {"block_bytes": block, "encode_s": t_enc[-1], "decode_s": t_dec[-1],
            "encode_GBps": enc_b / t_enc[-1] / 1e9,
            "decode_GBps": dec_b / t_dec[-1] / 1e9,
            "encdec_GBps": (enc_b + dec_b) / (t_enc[-1] + t_dec[-1]) / 1e9,
            "ok": bool(ok)}


def stream_rate(k, m, nbytes):
    """qi::fec::RsFnt::encode/decode_streams_vertical (the two-slot pinned
    pipeline) through its C view over memory streams of `nbytes` per
    fragment: istream reads + H2D + kernels + D2H + ostream writes."""
    import ctypes as C
    lib = qa.lib()
    f = qa.Fec(k, m, False)
    no = f.n_outputs
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(k)]
    outs = [np.zeros(nbytes, np.uint8) for _ in range(no)]
    cap = 64 + nbytes // 1024
    oor = np.zeros((no, cap), np.uint32)
    cnt = np.zeros(no, np.uint32)
    t_enc = []
    for _ in range(2):
        t = time.perf_counter()
        assert lib.qi_fec_encode_streams(
            f.h, qa.ptr_array(data), nbytes, qa.ptr_array(outs),
            oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
            cap) == 0
        t_enc.append(time.perf_counter() - t)
    missing = np.zeros(k + m, bool)
    missing[rng.choice(k + m, m, replace=False)] = True
    par = [None if missing[i] else outs[i] for i in range(no)]
    dec = [np.zeros(nbytes, np.uint8) for _ in range(k)]
    t_dec = []
    for _ in range(2):
        t = time.perf_counter()
        assert lib.qi_fec_decode_streams(
            f.h, None, qa.ptr_array(par), nbytes,
            oor.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
            cap, qa.ptr_array(dec)) == 1
        t_dec.append(time.perf_counter() - t)
    ok = all((dec[i] == data[i]).all() for i in range(k))
    enc_b, dec_b = alg_bytes(k, m, nbytes // 2)
    f.close()
    return {"bytes_per_fragment": nbytes, "encode_s": t_enc[-1],
            "decode_s": t_dec[-1],
            "encode_GBps": enc_b / t_enc[-1] / 1e9,
            "decode_GBps": dec_b / t_dec[-1] / 1e9,
            "encdec_GBps": (enc_b + dec_b) / (t_enc[-1] + t_dec[-1]) / 1e9,
            "ok": bool(ok)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=512)
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--cabi-block-mib", type=int, default=16)
    args = ap.parse_args()
    k, m, P = 16, 48, 32768
    S, Cn, NS = args.stripes, args.chunk, args.streams
    assert S % Cn == 0
    plan = qa.Plan(k, m, False)
    n = plan.n_outputs
    cap = 64
    rng = np.random.default_rng(7)

    h_data = torch.from_numpy(
        rng.integers(-32768, 32768, (S, k, P), dtype=np.int16)).pin_memory()
    h_coded = torch.empty((S, n, P), dtype=torch.int16, pin_memory=True)
    h_cnt = torch.empty((S, n), dtype=torch.int32, pin_memory=True)
    h_ent = torch.empty((S, n, cap), dtype=torch.int32, pin_memory=True)
    h_dec = torch.empty((S, k, P), dtype=torch.int16, pin_memory=True)
    streams = [torch.cuda.Stream() for _ in range(NS)]
    dev = [dict(data=torch.empty((Cn, k, P), dtype=torch.int16, device="cuda"),
                coded=torch.empty((Cn, n, P), dtype=torch.int16, device="cuda"),
                dec=torch.empty((Cn, k, P), dtype=torch.int16, device="cuda"),
                cnt=torch.empty((Cn, n), dtype=torch.int32, device="cuda"),
                ent=torch.empty((Cn, n, cap), dtype=torch.int32, device="cuda"),
                ids=torch.empty((Cn, k), dtype=torch.int16, device="cuda"),
                pcnt=torch.empty((Cn, k), dtype=torch.int32, device="cuda"),
                pent=torch.empty((Cn, k, cap), dtype=torch.int32, device="cuda"),
                ctx=torch.empty(plan.ctx_bytes(Cn, P), dtype=torch.uint8,
                                device="cuda"))
           for _ in range(NS)]

    def encode_all():
        for c in range(S // Cn):
            b, st = dev[c % NS], streams[c % NS]
            sl = slice(c * Cn, (c + 1) * Cn)
            with torch.cuda.stream(st):
                b["data"].copy_(h_data[sl], non_blocking=True)
                b["cnt"].zero_()
                plan.encode(b["data"], b["coded"], b["cnt"], b["ent"], cap,
                            stream=st.cuda_stream)
                h_coded[sl].copy_(b["coded"], non_blocking=True)
                h_cnt[sl].copy_(b["cnt"], non_blocking=True)
                h_ent[sl].copy_(b["ent"], non_blocking=True)
        torch.cuda.synchronize()

    encode_all()  # warm-up
    t0 = time.perf_counter()
    encode_all()
    t_enc = time.perf_counter() - t0

    # received fragments: a random k-subset per stripe, staged back to back
    # (what the network / file reader would deliver), not timed
    ids = np.sort(np.stack([rng.choice(k + m, k, replace=False)
                            for _ in range(S)]), axis=1)
    idx = torch.from_numpy(ids.astype(np.int64))
    h_recv = torch.gather(h_coded, 1, idx[:, :, None].expand(S, k, P)).pin_memory()
    h_pcnt = torch.gather(h_cnt, 1, idx).pin_memory()
    h_pent = torch.gather(h_ent, 1, idx[:, :, None].expand(S, k, cap)).pin_memory()
    h_ids = torch.from_numpy(ids.astype(np.int16)).pin_memory()

    def decode_all():
        for c in range(S // Cn):
            b, st = dev[c % NS], streams[c % NS]
            sl = slice(c * Cn, (c + 1) * Cn)
            with torch.cuda.stream(st):
                b["data"].copy_(h_recv[sl], non_blocking=True)
                b["ids"].copy_(h_ids[sl], non_blocking=True)
                b["pcnt"].copy_(h_pcnt[sl], non_blocking=True)
                b["pent"].copy_(h_pent[sl], non_blocking=True)
                plan.decode_ctx_packed(b["ids"], b["ctx"], P, b["pcnt"],
                                       b["pent"], cap, stream=st.cuda_stream)
                plan.decode_packed(b["ctx"], b["data"], b["dec"],
                                   b["pcnt"], b["pent"], cap,
                                   stream=st.cuda_stream, check=False)
                h_dec[sl].copy_(b["dec"], non_blocking=True)
        torch.cuda.synchronize()

    decode_all()
    t0 = time.perf_counter()
    decode_all()
    t_dec = time.perf_counter() - t0
    ok = bool(torch.equal(h_dec, h_data)) and plan.take_error() == 0

    enc_b, dec_b = alg_bytes(k, m, P)
    cabi = cabi_rate(k, m, args.cabi_block_mib << 20)
    streams = stream_rate(k, m, 64 << 20)
    out = {
        "what": "host-inclusive RS-FNT k=16 n=64 pkt=64KiB (pinned host "
                "buffers, H2D + kernels + D2H, chunked over streams)",
        "stripes": S, "chunk_stripes": Cn, "streams": NS,
        "h2d_GBps": copy_rate(256 << 20, True),
        "d2h_GBps": copy_rate(256 << 20, False),
        "encode_ms_per_stripe": t_enc / S * 1e3,
        "decode_ms_per_stripe": t_dec / S * 1e3,
        "encode_GBps": S * enc_b / t_enc / 1e9,
        "decode_GBps": S * dec_b / t_dec / 1e9,
        "encdec_GBps": S * (enc_b + dec_b) / (t_enc + t_dec) / 1e9,
        "pcie_bytes_per_stripe": {"h2d": (k + k) * 2 * P,
                                  "d2h": (n + k) * 2 * P},
        "roundtrip_ok": ok and cabi.pop("ok") and streams.pop("ok"),
        "cabi": cabi,
        "streams": streams,
    }
    print(json.dumps(out))
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
