"""The generated rv32im accumulation kernels, run from their HIP source text by a numpy
interpreter of the emitted C subset (tests/gen_src_eval.py), equal the IR interpreter
(tests/rv32im_accum_ir.py, itself pinned to the compiled reference's stepAccum) on random
rows over all 13 instruction arms: the generator's rewrites — inverse batches, depth-first
emission with split guarded stores, load look-ahead, kernel cuts — keep the program's
meaning, checked on the CPU for the build's settings and for the unbatched program-order
baseline."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import gen_src_eval as GS
import rv32im_accum_ir as IRI
from test_rv32im_accum_ir import rows_for_arms

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _generate(tmp, limit, inv_batch, ahead, extra=()):
    out = os.path.join(tmp, f"rv_{limit}_{inv_batch}_{ahead}_{'_'.join(map(str, extra))}")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_accum.py"), "rv32im", out,
                           str(limit), str(inv_batch), str(ahead)] + [str(x) for x in extra],
                          stdout=subprocess.DEVNULL)
    launcher = open(os.path.join(out, "accum.hip")).read()
    order = re.findall(r"rv_accum::launch_k(\d+)\(s, A\);", launcher)
    return [open(os.path.join(out, f"accum_k{k}.hip")).read() for k in order]


# (limit, inv batch, look-ahead, [fuse, pack, sort]): the build's settings (fused sums,
# arm-sorted kernels packed to 20000), the fused contiguous cut, the unfused one, and the
# unbatched program-order baseline
@pytest.mark.parametrize("limit,inv_batch,ahead,extra", [(1200, 8, 64, ()), (1200, 8, 64, (1, 0, 0)),
                                                         (1200, 8, 64, (0, 0, 0)), (1200, 1, 0, (0, 0, 0)),
                                                         (600, 16, 0, (1, 8000, 256))])
@pytest.mark.parametrize("rows,last", [(64, 64), (64, 50)])
def test_generated_source_matches_ir(tmp_path, limit, inv_batch, ahead, extra, rows, last):
    kernels = _generate(str(tmp_path), limit, inv_batch, ahead, extra)
    rng = np.random.default_rng(rows + last + limit + inv_batch)
    data = rows_for_arms(rng, rows, list(rng.integers(0, 13, rows)))
    glob = rng.integers(0, GS.P, 90, dtype=np.uint64).astype(np.uint32)
    mix = rng.integers(0, GS.P, 36, dtype=np.uint64).astype(np.uint32)
    want = np.full(103 * rows, 0xFFFFFFFF, np.uint32)
    IRI.run(data.copy(), want, glob, mix, rows, last)
    got = np.full(103 * rows, 0xFFFFFFFF, np.uint32)
    bufs = [data.copy(), got, glob, mix]
    for src in kernels:
        GS.run_kernel(src, bufs, rows, last)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} words differ; first at col {bad[0] // rows} row {bad[0] % rows}"
    if inv_batch > 1:
        assert any("fp_inv_batch" in k for k in kernels)


def _generate_recursion(tmp, ahead):
    out = os.path.join(tmp, f"rec_{ahead}")
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_accum.py"), "recursion", out,
                           "1200", "8", str(ahead)], stdout=subprocess.DEVNULL)
    launcher = open(os.path.join(out, "accum.hip")).read()
    fns = {}
    for name, body in re.findall(r"void recursion_accum_(\w+)\(hipStream_t s, const AccArgs& A\) \{(.*?)\}",
                                 launcher, re.S):
        fns[name] = [open(os.path.join(out, f"accum_k{k}.hip")).read()
                     for k in re.findall(r"launch_k(\d+)\(s, A\);", body)]
    return fns


@pytest.mark.parametrize("ahead", [64, 0])
def test_generated_recursion_source_matches_ir(tmp_path, oracle, ahead):
    """Recursion: compute kernels, the FpExt prefix product, verify kernels, from source,
    equal tests/accum_ir.py's interpretation of the IR (pinned to the compiled reference)."""
    import accum_ir as A
    fns = _generate_recursion(str(tmp_path), ahead)
    d = A.circuit()
    gs = d["group_sizes"]
    po2 = 6
    n = 1 << po2
    steps = n - 3
    rng = np.random.default_rng(77 + ahead)
    ctrl, glob, data, mix = A.synthetic(rng, oracle, po2, gs, d["output_size"], d["mix_size"])
    acc0 = np.full(gs[0] * n, 0xFFFFFFFF, np.uint32)
    want = A.accum(ctrl, glob, data, mix, acc0, steps, n)
    got = acc0.copy()
    bufs = [ctrl, glob, data, mix, got]
    vals = np.zeros((steps, 4), np.int64)
    vals[:, 0] = GS.R
    for src in fns["compute"]:
        GS.run_kernel(src, bufs, n, steps, vals)
    acc = [1, 0, 0, 0]
    for c in range(steps):  # the inclusive product scan, on plain values
        acc = A._emul(acc, [int(x) * GS.RINV % GS.P for x in vals[c]])
        vals[c] = [x * GS.R % GS.P for x in acc]
    for src in fns["verify"]:
        GS.run_kernel(src, bufs, n, steps, vals)
    assert np.array_equal(got, want), int((got != want).sum())
