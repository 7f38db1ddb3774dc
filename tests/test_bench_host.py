"""bench.py's host-side choices (no GPU): which committed PMC summary the roofline quotes."""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _summaries(tmp_path, tags, lib_of):
    prof = tmp_path / "profiles"
    prof.mkdir()
    for t in tags:
        doc = {"kernels": {}, "per_proof": {}}
        if t in lib_of:
            doc["lib_sha256_16"] = lib_of[t]
        (prof / f"{t}_pmc_valu.json").write_text(json.dumps(doc))
    return prof


def test_pmc_summary_round_order(tmp_path, monkeypatch):
    # r5an is newer than r5v (tag length first), r5a newer than r4x: plain string order gets both wrong
    _summaries(tmp_path, ["r4x", "r5a", "r5v", "r5z", "r5aa", "r5an"], {})
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_fingerprint", lambda: "0123456789abcdef")
    assert os.path.basename(bench.pmc_summary_file("valu")) == "r5an_pmc_valu.json"
    assert bench.pmc_summary_file("traffic") is None


def test_pmc_summary_prefers_loaded_library(tmp_path, monkeypatch):
    _summaries(tmp_path, ["r5p", "r5v", "r5an"], {"r5p": "aaaa", "r5v": "bbbb", "r5an": "cccc"})
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_fingerprint", lambda: "bbbb")
    assert os.path.basename(bench.pmc_summary_file("valu")) == "r5v_pmc_valu.json"
    monkeypatch.setattr(bench, "lib_fingerprint", lambda: "dddd")
    assert os.path.basename(bench.pmc_summary_file("valu")) == "r5an_pmc_valu.json"
