"""The sampled full-size eval_check checker (oracle.eval_check_sampled, used by the -m gpu
full-size parity tests at po2 20/24) equals the whole-domain oracle eval_check
(rv32im/src/prove/hal/cpu.rs:145-207 with the reference's compiled poly_fp) at every
cycle of a small domain, including the back-wrap cycles 0 .. 4*68."""
import numpy as np
import pytest


def test_splitmix_fill_offsets(oracle):
    a = oracle.splitmix_fill(7, 1000)
    assert np.array_equal(a[300:], oracle.splitmix_fill(7, 700, start=300))
    assert a.max() < oracle.P


@pytest.mark.parametrize("circuit,po2", [("rv32im", 7), ("recursion", 7)])
def test_sampled_eval_check_equals_full(oracle, circuit, po2):
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    d = oracle.load_circuit_json(circuit)
    D = 4 << po2
    seeds = [0x1111 + po2, 0x2222 + po2, 0x3333 + po2]
    groups = [oracle.splitmix_fill(seeds[g], d["group_sizes"][g] * D) for g in range(3)]
    rng = np.random.default_rng(po2)
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    full = np.zeros(4 * D, np.uint32)
    oracle.eval_check(circuit, full, groups, mix, glob, pm, po2)
    cycles = np.arange(D, dtype=np.uint64)
    got = oracle.eval_check_sampled(circuit, seeds, mix, glob, pm, po2, cycles)
    assert np.array_equal(got.T, full.reshape(4, D))
