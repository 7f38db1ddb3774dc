"""World-size-2 CPU rehearsal of the segment-per-GPU path (risc0_amd/segments.py, SURVEY.md
§8e): the local launcher (what `bench.py --gpus N` uses without torch.distributed.run)
starts 2 gloo ranks; each proves its round-robin share of the golden seal cases with the
CPU oracle; rank 0 gathers the seal digests host-side and they equal the golden fixtures
(tests/golden/index.json), with the reported time the max over ranks."""
import json
import os
import sys

import pytest

from risc0_amd.segments import launch_local, rank_env, segments_for_rank

HERE = os.path.dirname(os.path.abspath(__file__))


def test_round_robin_covers_all_segments():
    for world in (1, 2, 3, 8):
        got = sorted(s for r in range(world) for s in segments_for_rank(r, world, 64))
        assert got == list(range(64))


def test_rank_env_matches_torchrun():
    e = rank_env(3, 8, 29500, base={})
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"]) == \
        ("3", "3", "8", "127.0.0.1", "29500")


def test_rank_binds_one_device_like_r0vm():
    """Each rank sees only its own GPU, as r0vm's workers do (CUDA_VISIBLE_DEVICES=idx,
    r0vm/src/actors/mod.rs:449-462), and opens it as ordinal 0."""
    from risc0_amd.segments import narrow_visible_devices
    assert rank_env(3, 8, 1, base={})["HIP_VISIBLE_DEVICES"] == "3"
    # an inherited list is indexed by the local rank
    assert rank_env(1, 2, 1, base={"HIP_VISIBLE_DEVICES": "4,6"})["HIP_VISIBLE_DEVICES"] == "6"
    e = rank_env(2, 4, 1, base={"CUDA_VISIBLE_DEVICES": "0,1,2,3"})
    assert e["HIP_VISIBLE_DEVICES"] == "2" and "CUDA_VISIBLE_DEVICES" not in e
    # the child (bench.py) binds again: already bound, it keeps its one device, ordinal 0
    assert narrow_visible_devices(2, e) == 0 and e["HIP_VISIBLE_DEVICES"] == "2"
    # torch.distributed.run ranks (no launch_local) bind themselves
    env = {"LOCAL_RANK": "5"}
    assert narrow_visible_devices(5, env) == 0 and env["HIP_VISIBLE_DEVICES"] == "5"
    # more ranks than inherited devices: shared round-robin, flagged for the bench line
    short = {"HIP_VISIBLE_DEVICES": "0,1"}
    assert narrow_visible_devices(2, short) == 0 and short["HIP_VISIBLE_DEVICES"] == "0"
    assert short["R0_RANKS_SHARE_DEVICES"] == "1"
    with pytest.raises(RuntimeError):
        narrow_visible_devices(0, {"HIP_VISIBLE_DEVICES": ","})
    # the rehearsal switch leaves the devices to bench.py's round-robin
    assert "R0_RANK_BOUND" not in rank_env(1, 2, 1, base={"HIP_VISIBLE_DEVICES": "0", "R0_BENCH_SHARE_GPUS": "1"})


@pytest.mark.timeout(300)
def test_two_ranks_prove_golden_segments(oracle, tmp_path):
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    import test_golden as G
    out = tmp_path / "dist.json"
    rc = launch_local(2, [sys.executable, os.path.join(HERE, "dist_worker.py"), str(out)], timeout=280)
    assert rc == 0
    res = json.loads(out.read_text())
    cases = G.INDEX["seals"]
    assert res["world"] == 2
    assert {int(k) for k in res["digests"]} == set(range(len(cases)))
    for k, d in res["digests"].items():
        assert d == cases[int(k)]["seal_sha256"], f"segment {k} seal differs from its golden digest"
    assert abs(res["tmax"] - max(res["t_by_rank"].values())) < 1e-9
