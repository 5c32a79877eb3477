"""CPU: the compiler's resource report of the gfx950 kernels
(build/obj/{kernels,ctx,ntt}.res, written by quadiron_amd/csrc/Makefile).  A hot kernel
that spills to scratch memory runs through memory instead of registers (a
y[16] epilogue array once landed there and doubled the decode time), so
scratch use is an error outside the listed rare paths."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RES = [os.path.join(ROOT, "build", "obj", f)
       for f in ("kernels.res", "ctx.res", "ntt.res")]

# kernels allowed to use scratch: the adversarial-OOR recompute and the
# K = 64 encode codelet (256 VGPRs at 2 waves/SIMD, 3-4 spilled registers;
# 3 waves/SIMD spilled 280 and ran 20 % slower, profiles/r1_ab_k64_encode.txt)
# (the dot2 column tails of k > 64, matrix_kernel<64|128>, no longer spill:
# their 128-256 row ids are read from VGPR lanes instead of SGPRs)
# Round 6: the k > 128 decode context (1024 threads, 128 VGPRs: a few values
# kept across the chunk loop, 5 reloads per chunk; the non-systematic k300 /
# k600 contexts measured 48 / 102 us either way, gpurun_out/r6k).
ALLOWED = ("matrix_redo_kernel", "encode_fnt_kernelILi64E",
           "decode_ctx_kernelILi1024ELb1E")


def kernels():
    if not all(os.path.exists(r) for r in RES):
        pytest.skip("kernel resource report not built (make -C quadiron_amd/csrc)")
    out, cur = {}, None
    for line in (ln for r in RES for ln in open(r)):
        m = re.search(r"remark: (?:\S+:\d+:\d+: )?Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark: (?:\S+:\d+:\d+: )?\s*([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur:
            out[cur][m.group(1).strip()] = int(m.group(2))
    return out


def test_report_lists_the_hot_kernels():
    ks = kernels()
    for name in ("encode_fnt_kernel", "matrix_mfma_kernel", "matrix_kernel",
                 "decode_ctx_kernel", "matrix_redo_kernel", "ntt_pass_kernel",
                 "ntt_ctx_kernel", "ntt_expand_kernel", "ntt_fix_kernel"):
        assert any(name in k for k in ks), name


def test_no_scratch_in_hot_kernels():
    bad = {k: v.get("ScratchSize") for k, v in kernels().items()
           if v.get("ScratchSize", 0) > 0 and not any(a in k for a in ALLOWED)}
    assert not bad, bad


def _lds_waves_per_simd(ks, nst, rsplit):
    """Waves per SIMD the matrix-core kernel's LDS allows (MfmaTile: image
    2 * 16 KS rows of 64 NST + 16 bytes, mark list, per-wave staging tiles
    when it has several row blocks; 4 waves per block, 160 KiB per CU)."""
    img = 2 * 16 * ks * (64 * nst + 16)
    lds = img + 2 * 4 * 256 + 16 + (4 * 16 * 144 if rsplit or ks > 1 else 0)
    return min(8, (160 * 1024) // lds)


def test_mfma_kernel_occupancy():
    """The matrix-core kernels keep the occupancy their LDS image allows
    (registers must not be the tighter limit), and at least 2 waves per
    SIMD."""
    for k, v in kernels().items():
        m = re.search(r"matrix_mfma_kernelILi(\d+)ELi(\d+)ELi4ELb(\d)E", k)
        if not m:
            continue
        ks, nst, rsplit = int(m.group(1)), int(m.group(2)), m.group(3) == "1"
        want = max(2, min(4, _lds_waves_per_simd(ks, nst, rsplit)))
        if ks >= 8:
            want = 2  # 128 < 16 KS rows: 198-248 VGPRs
        assert v.get("Occupancy", 0) >= want, (k, v, want)
