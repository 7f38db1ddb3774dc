"""One rank of the world-size-N CPU rehearsal of the segment-per-GPU harness
(tests/test_segments_dist.py): started by risc0_amd.segments.launch_local with the
torch.distributed.run environment, it proves its round-robin share of the golden seal
cases with the CPU oracle (the GPU's stand-in here), gathers seal digests host-side and
rank 0 writes the result as JSON to argv[1]."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE, os.path.join(ROOT, "oracle")]


def main(out_path):
    import torch.distributed as dist

    import oracle
    import test_golden as G
    from risc0_amd.segments import gather_results, segments_for_rank, timed_segments
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # launch_local bound this rank to one device (r0vm's CUDA_VISIBLE_DEVICES=idx)
    assert os.environ["HIP_VISIBLE_DEVICES"] == str(rank) and os.environ["R0_RANK_BOUND"] == "1"
    dist.init_process_group("gloo", init_method="env://")
    cases = G.INDEX["seals"]
    suites = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}
    mine = segments_for_rank(rank, world, len(cases))
    digests = {}

    def prove(seg):
        c = cases[seg]
        w = G.seal_inputs(oracle, c["circuit"], c["po2"])
        seal, _mix, _ = oracle.prove_segment(c["circuit"], suites[c["suite"]], c["po2"], *w,
                                             version=2 if c["circuit"] == "rv32im" else None)
        digests[seg] = G.digest(seal)

    t, tmax = timed_segments(prove, mine, 0, lambda: None, dist)
    ts = gather_results({rank: t}, dist)
    got = gather_results(digests, dist)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump({"digests": {str(k): v for k, v in got.items()}, "t_by_rank": ts, "tmax": tmax,
                       "world": world, "env_ranks": os.environ["LOCAL_RANK"]}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
