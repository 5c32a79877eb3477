"""CPU: the product library builds, loads, and exports every entry point the
public headers declare (no compute calls -- there is no GPU here)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["quadiron_c.h", "qi_gpu.h"]


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src)
    kw = {"if", "sizeof", "defined", "return"}
    return sorted({n for n in names if n not in kw and
                   (n.startswith("quadiron_") or n.startswith("qi_"))})


@pytest.mark.parametrize("header", HEADERS)
def test_library_exports_header_symbols(header):
    import quadiron_amd
    lib = quadiron_amd.lib()
    names = declared(header)
    assert len(names) >= 5
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_dropin_abi_matches_reference_names():
    # exactly the seven entry points of src/quadiron_c.h:34-160
    assert declared("quadiron_c.h") == sorted([
        "quadiron_fnt32_new", "quadiron_fnt32_delete",
        "quadiron_fnt32_get_metadata_size", "quadiron_fnt32_encode",
        "quadiron_fnt32_decode", "quadiron_fnt32_reconstruct",
        "quadiron_hex_dump"])


def test_no_device_is_reported_not_faked():
    """Without a GPU the library must refuse work, not fall back to CPU."""
    import quadiron_amd
    lib = quadiron_amd.lib()
    if lib.qi_gpu_device_count() > 0:
        pytest.skip("a device is visible")
    assert lib.qi_plan_create(16, 48, 0) is None
    assert lib.quadiron_fnt32_new(2, 16, 48, 0) is None
    with pytest.raises(RuntimeError):
        quadiron_amd.Plan(16, 48)
