"""The Rust binding a maintainer adds (integration/rust/sys_hip.rs)
declares every r0hip_* entry point of include/r0hip.h with the same number of
parameters. The Rust sources are not compiled here (no Rust toolchain in the image)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _params(text, name, lang):
    m = re.search(r"\b" + name + r"\s*\(", text)
    assert m, f"{name} not declared ({lang})"
    depth, i = 1, m.end()
    start = i
    while depth:
        depth += {"(": 1, ")": -1}.get(text[i], 0)
        i += 1
    body = text[start:i - 1].strip().rstrip(",").strip()
    if body in ("", "void"):
        return 0
    return body.count(",") + 1


def test_rust_sys_binding_covers_the_c_abi():
    hdr = open(os.path.join(ROOT, "include", "r0hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    rs = open(os.path.join(ROOT, "integration", "rust", "sys_hip.rs")).read()
    rs = re.sub(r"//[^\n]*", "", rs)
    names = sorted(set(re.findall(r"\b(r0hip_\w+)\s*\(", hdr)))
    assert len(names) > 40
    for n in names:
        assert _params(hdr, n, "C") == _params(rs, n, "Rust"), n


def test_rust_hal_implements_every_hal_method():
    """hal_hip.rs implements each method of risc0_zkp::hal::Hal (hal/mod.rs:55-258) that the
    Python mirror (risc0_amd.HipHal) exposes."""
    rs = open(os.path.join(ROOT, "integration", "rust", "hal_hip.rs")).read()
    methods = ["has_unified_memory", "get_hash_suite", "alloc_digest", "alloc_elem", "alloc_extelem", "alloc_u32",
               "alloc_elem_init", "alloc_extelem_zeroed", "copy_from_digest", "copy_from_elem", "copy_from_extelem",
               "copy_from_u32", "batch_expand_into_evaluate_ntt", "batch_interpolate_ntt", "batch_bit_reverse",
               "batch_evaluate_any", "zk_shift", "mix_poly_coeffs", "eltwise_add_elem", "eltwise_sum_extelem",
               "eltwise_copy_elem", "eltwise_copy_elem_slice", "eltwise_zeroize_elem", "fri_fold", "hash_rows",
               "hash_fold", "gather_sample", "scatter", "prefix_products", "combos_prepare", "combos_divide"]
    for m in methods:
        assert re.search(r"fn " + m + r"\b", rs), m


def test_rust_recursion_circuit_hal_binds_the_recursion_entry_points():
    """recursion_circuit_hal_hip.rs (circuit/recursion/src/prove/hal/hip.rs, beside the
    reference's cuda.rs) implements the recursion circuit's three HAL traits over the C ABI"""
    rs = open(os.path.join(ROOT, "integration", "rust", "recursion_circuit_hal_hip.rs")).read()
    for trait in ("CircuitWitnessGenerator", "CircuitAccumulator", "CircuitHal"):
        assert re.search(r"impl<HS: HipHash> " + trait + r"<HipHal<HS>> for HipRecursionCircuitHal<HS>", rs), trait
    for sym in ("r0hip_recursion_witgen", "r0hip_recursion_accum", "r0hip_eval_check"):
        assert re.search(sym + r"\(", rs), sym
    for suite in ("HipHashPoseidon2", "HipHashPoseidon254", "HipHashSha256"):
        assert suite in rs
    # the rv32im circuit HAL no longer carries it as comments
    rv = open(os.path.join(ROOT, "integration", "rust", "circuit_hal_hip.rs")).read()
    assert "HipRecursionCircuitHal" not in rv.replace("recursion_circuit_hal_hip.rs", "")


def test_rust_hal_node_heap_mirror_is_invalidated_by_every_digest_write():
    """hal_hip.rs answers get_at on a Merkle node heap from a host mirror (one bulk copy per
    tree instead of one synchronous copy per node). The Hal methods that write a Buffer<Digest>
    are hash_rows and hash_fold (hal/mod.rs:55-258), plus Buffer::view_mut: each must clear the
    mirror, and hash_fold's root layer starts the heap's mirror copy."""
    rs = open(os.path.join(ROOT, "integration", "rust", "hal_hip.rs")).read()

    def body(name):
        m = re.search(r"fn " + name + r"\b[^{]*\{", rs)
        assert m, name
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(rs[i], 0)
            i += 1
        return rs[m.end():i]
    assert "io.written(output_size == 1)" in body("hash_fold")
    assert "output.written(false)" in body("hash_rows")
    assert "self.written(false)" in body("view_mut")
    # no other Hal method takes a Buffer<Digest>
    sigs = re.findall(r"fn (\w+)\([^)]*Buffer<Digest>", rs)
    assert set(sigs) <= {"hash_rows", "hash_fold", "alloc_digest", "copy_from_digest"}, sigs
