"""CPU-only checks of the drop-in boundary: the C-ABI library loads and exports every
entry point include/r0hip.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    import risc0_amd as r
    L = r.lib()
    declared = r.exported_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing


def test_exports_are_c_linkage():
    lib = os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so")
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib]).decode()
    syms = set(re.findall(r"\bT (r0hip_\w+)", out))
    import risc0_amd as r
    assert set(r.exported_symbols()) <= syms


def test_library_is_gfx950_only():
    """every device code object in the library's offload bundles targets gfx950 (hipcub's
    host code names other architectures in its tuning tables; those are strings, not code)"""
    lib = os.path.join(ROOT, "risc0_amd", "lib", "libr0hip.so")
    data = open(lib, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets
    assert b"nvptx" not in data


def test_errors_are_reported_not_fatal():
    # without a visible device, init must return an error string (no abort)
    import risc0_amd as r
    if os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"):
        return  # a GPU may be present; covered by the gpu tests
    err = r.lib().r0hip_init(0)
    assert err  # message, not a crash
    r.lib().r0hip_free_error(err)
