"""configs[3]'s input on the CPU: one loop.s session cut into consecutive segments
(rv32im_trace.LoopSession). The segments chain (each pre-state root is the previous post-state
root, each resumes from the previous final memory mid-loop), fill their segments to the
executor's split, the compiled reference witgen accepts each, and a continuation segment's
CPU-path seal (compiled reference witgen + accumulation around the oracle prover) passes the
native verifier with the validity equation."""
import numpy as np

import rv32im_trace as T
import rv32im_witgen_ref as W


def test_loop_s_session_chains_and_verifies(oracle):
    import risc0_amd as r
    po2, K = 15, 3
    S = T.LoopSession(po2, T.loop_s_session_iterations(po2, K), seed=5)
    traces = list(S)
    assert len(traces) == K and traces[-1].terminated
    for a, b in zip(traces, traces[1:]):
        assert b.root == a.post_root
        # resumes in user mode inside the loop, counter carried over
        assert b.final_mem is not a.final_mem
    for t in traces[:-1]:
        assert t.table_split_cycle + T.RESERVED_CYCLES >= (1 << po2) - 2 * T.LoopSession.MARGIN
    for t in traces:
        W.witgen(t, W.MODE_PARALLEL)  # raises with the reference's message if the trace is refused
    seal, mix, *_ = W.prove_from_trace(traces[1], oracle.POSEIDON2, oracle)
    assert r.verify_seal("rv32im", r.POSEIDON2, seal, check_validity=True) == po2


def test_loop_s_session_fast_forward_matches_building():
    """segment(k) with the earlier segments fast-forwarded (executor pass only) gives the same
    trace as building every segment in order"""
    po2, K = 15, 3
    it = T.loop_s_session_iterations(po2, K)
    built = list(T.LoopSession(po2, it, seed=7))
    skipped = T.LoopSession(po2, it, seed=7).segment(2)
    a, b = built[2], skipped
    assert a.root == b.root and a.post_root == b.post_root
    for x, y in zip(a.arrays(), b.arrays()):
        assert np.array_equal(x, y)
    for x, y in zip(a.injector_arrays(), b.injector_arrays()):
        assert np.array_equal(x, y)
