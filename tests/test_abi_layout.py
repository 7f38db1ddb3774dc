"""The ctypes mirrors in risc0_amd/hal.py have the layout of the C structs they stand for in
include/r0hip.h: a small C program, compiled here with gcc against the header, prints sizeof and
every field's offsetof, and each must equal the ctypes Structure's. A drift (a field added on one
side only, as round 6 did to r0hip_trace_job) would otherwise show up only as garbage on a GPU."""
import ctypes as C
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mirrors():
    from risc0_amd import hal
    return {
        "r0hip_bigint_back": hal.BigIntBack,
        "r0hip_raw_buffer": hal.RawBuffer,
        "r0hip_raw_exec_buffers": hal.RawExecBuffers,
        "r0hip_raw_preflight_trace": hal.RawPreflightTrace,
        "r0hip_trace_input": hal.TraceInput,
        "r0hip_segment_job": hal.SegmentJob,
        "r0hip_trace_job": hal.TraceJobStruct,
    }


# ctypes field names that differ from the C ones (`global` is a Python keyword)
C_NAME = {("r0hip_raw_exec_buffers", "glob"): "global"}


def test_ctypes_structs_match_the_c_header():
    mirrors = _mirrors()
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "r0hip.h"', "int main(void) {"]
    for cname, py in mirrors.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            cf = C_NAME.get((cname, f[0]), f[0])
            lines.append(f'  printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {cf}));')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "layout.c"), os.path.join(d, "layout")
        with open(src, "w") as fh:
            fh.write("\n".join(lines))
        cc = subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), src, "-o", exe],
                            capture_output=True, text=True)
        if cc.returncode:
            pytest.fail("the header does not compile as C with these field names:\n" + cc.stderr)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            cname, field, val = ln.split()
            got[(cname, field)] = int(val)
    for cname, py in mirrors.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for f in py._fields_:
            assert got[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])


def _c_fields(hdr, cname):
    import re
    m = re.search(r"typedef struct " + cname + r" \{(.*?)\} " + cname + ";", hdr, flags=re.S)
    assert m, cname
    body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
    return [re.search(r"(\w+)\s*(\[\d+\])?\s*$", d.strip()).group(1) for d in body.split(";") if d.strip()]


def test_rust_ffi_structs_have_the_header_fields_in_order():
    """integration/rust/sys_hip.rs declares the #[repr(C)] structs with the header's fields in
    the header's order (their types are checked by the Rust compiler where one exists)."""
    import re
    hdr = open(os.path.join(ROOT, "include", "r0hip.h")).read()
    rs = open(os.path.join(ROOT, "integration", "rust", "sys_hip.rs")).read()
    for rname, cname in (("R0HipBigIntBack", "r0hip_bigint_back"), ("R0HipTraceInput", "r0hip_trace_input"),
                         ("R0HipSegmentJob", "r0hip_segment_job"), ("R0HipTraceJob", "r0hip_trace_job")):
        m = re.search(r"pub struct " + rname + r" \{(.*?)\n\}", rs, flags=re.S)
        assert m, rname
        rfields = re.findall(r"pub (\w+):", m.group(1))
        assert rfields == _c_fields(hdr, cname), rname
