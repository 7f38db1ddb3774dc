#!/usr/bin/env python3
"""Group a rocprofv3 kernel_stats.csv by the launcher families that bench.py's
HIP-event timer reports (one launcher = several kernels, e.g. eval_check = the
generated ec_<circuit>::k<i> sequence), per proof: total ms / number of proofs.

  python tools/rocprof_families.py gpurun_out/.../run_kernel_stats.csv PROOFS
"""
import csv
import re
import sys

FAMILIES = [
    (r"ec_rv32im::k\d+|ec_recursion::k\d+", "eval_check"),
    (r"p2_rows_kernel|sha_rows_kernel", "hash_rows"),
    (r"p2_fold_kernel|p2_fold2_kernel|p2_fold_quad_kernel|sha_fold_kernel|fold_top_kernel|p254_fold_kernel", "merkle_fold"),
    (r"ntt_pass_kernel<false", "ntt_evaluate"),
    (r"ntt_pass_kernel<true", "ntt_interpolate"),
    (r"bit_reverse", "bit_reverse"),
    (r"eval_any|eval_chunk|eval_tables", "batch_evaluate_any"),
    (r"mix_kernel", "mix_poly_coeffs"),
    (r"div_", "poly_divide"),
    (r"rvwg::witgen_major_|bucket_count_kernel|bucket_fill_kernel|rocprim::", "rv32im_witgen"),
    (r"rv_accum::|tile_sums_kernel|scan_sums_kernel|tile_scan_kernel|finalize_kernel|bigint_scatter_kernel",
     "rv32im_accum"),
]


def family(name):
    for pat, fam in FAMILIES:
        if re.search(pat, name):
            return fam
    return re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))[:50]


def main(path, proofs):
    agg = {}
    for r in csv.DictReader(open(path)):
        f = family(r["Name"])
        ms, n = agg.get(f, (0.0, 0))
        agg[f] = (ms + float(r["TotalDurationNs"]) / 1e6, n + int(r["Calls"]))
    total = sum(v[0] for v in agg.values())
    print(f"{'family':28s} {'ms/proof':>9s} {'launches/proof':>15s} {'share':>6s}")
    for f, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{f:28s} {ms / proofs:9.3f} {n / proofs:15.1f} {100 * ms / total:5.1f}%")
    print(f"{'TOTAL':28s} {total / proofs:9.3f}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]))
