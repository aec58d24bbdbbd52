"""CPU-side checks of the C ABI: the in-tree library loads and exports every symbol the header
declares (no compute calls: there is no GPU in the build container)."""
import ctypes
import os
import re

from adipose_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "adipose_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(adp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    lib = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"missing export {s}"
    assert set(syms) == set(_lib.exported_symbols()), "ctypes signature table out of sync with the header"


def test_abi_version_and_error_plumbing():
    lib = _lib.lib()
    assert lib.adp_abi_version() == _lib.ABI_VERSION == 21
    assert isinstance(lib.adp_last_error(), bytes)


def test_conv_desc_layout_matches_header():
    # 15 ints, float, uint, 6 ints, float, int, float, int, int, int (out_fp8), int (bn_defer_fold)
    # -> 30 4-byte fields
    assert ctypes.sizeof(_lib.ConvDesc) == 33 * 4
    # 16 operand pointers + 7 fused BatchNorm-backward reduction pointers + fp8 weight scales + act_outA (v18)
    assert ctypes.sizeof(_lib.ConvIO) == 25 * 8


CLIENT = os.path.join(ROOT, "adipose_tissue-unet_amd", "abi_client")


def test_c_client_links_and_reports_errors():
    """tests/c_abi/abi_client.c, a plain C11 caller of the handle ABI built by the library's Makefile (gcc against
    libadipose_hip.so and the HIP runtime): it links, sees the header's ABI version, and gets a status code and a
    message from adp_create for an unknown preset -- no device needed."""
    import subprocess
    if not os.path.exists(CLIENT):
        subprocess.run(["make", "-C", os.path.join(ROOT, "adipose_tissue-unet_amd", "csrc")], check=True,
                       capture_output=True)
    r = subprocess.run([CLIENT, "nogpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "nogpu: 0 failed" in r.stdout
