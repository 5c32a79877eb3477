"""The kernel names a plan reports (qi_gpu_kernels, carried by every bench
line and matched against rocprofv3's kernel statistics) must be kernels the
library actually contains, spelled as the demangler spells them -- a name
that is not an instantiation of the loaded library is a wrong bench line."""
import subprocess

import pytest

import bench

pytestmark = pytest.mark.gpu


def _kernel_symbols(path):
    out = subprocess.run(["nm", "-DC", path], check=True, capture_output=True,
                         text=True).stdout
    return [ln.split(" ", 2)[2] for ln in out.splitlines() if " qi::" in ln]


def _names(kernels):
    """'encode=a + b; decode=c + d (tail)' -> (role, name) pairs."""
    for part in kernels.split("; "):
        role, names = part.split("=", 1)
        for n in names.split(" + "):
            yield role, n.replace(" (tail)", "").strip()


@pytest.mark.parametrize("cfg,sys_", [
    ("cfg2", False), ("cfg2", True), ("cfg3", False), ("cfg1", False),
    ("k32", False), ("k128", False), ("k200", False), ("k256", False),
    ("k300", False), ("k384", False), ("k1000", False), ("k600", False),
    ("k600", True),
])
def test_reported_kernels_exist(cfg, sys_):
    import quadiron_amd as qa
    k, m, pkt, _ = bench.CONFIGS[cfg]
    plan = qa.Plan(k, m, sys_)
    syms = _kernel_symbols(qa.LIB_PATH)
    kernels = plan.kernels(pkt // 2)
    seen = {"encode": 0, "decode": 0}
    for role, name in _names(kernels):
        pre = "qi::" + name + ("(" if name.endswith(">") else "")
        assert any(pre in s for s in syms), (cfg, name, kernels)
        seen[role] += 1
    assert seen["encode"] >= 1 and seen["decode"] >= 2, kernels
    # the decode names its context builder first
    dec = kernels.split("; ")[1]
    assert "ctx_" in dec.split(" + ")[0] or dec.startswith("decode=ntt_ctx_kernel")

    # 256 < k <= 640 at whole-tile widths: the NTT engine's context is built
    # only by a decode the matrix cores cannot take; the
    # k600 decode runs the matrix cores at KS = 40 (round 6)
    if cfg in ("k300", "k384", "k600"):
        assert "ntt_ctx_kernel" not in dec, kernels
    if cfg == "k600":
        two = "true" if sys_ else "false"
        assert f"matrix_os_kernel<40, 8, 1, {two}>" in dec, kernels
