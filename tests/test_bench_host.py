"""bench.py host logic on CPU: the workloads build with the shapes
BASELINE.json names, the FLOP accounting matches the
survey's per-frame figures, and the default (headline) workload has a
committed PMC traffic summary of its own kernel shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_workload_shapes():
    expect = {"lidar": ([32400], "CmtLidarHead", 900), "fusion": ([56400], "CmtHead", 900),
              "coop": ([36400, 44400], "CmtHeadCoop", 900), "stress4": ([48400] * 4, "CmtHeadCoop", 1500)}
    for name, (nks, cls, nq) in expect.items():
        head, cfg, fwd, got, oracle_fwd = bench.make_workload(name, seed=0)
        assert got == nks, name
        assert type(head).__name__ == cls
        assert head.num_query == nq and head.transformer.decoder.num_layers == 6
        assert callable(fwd) and callable(oracle_fwd)


def test_default_workload_is_the_headline_config():
    import argparse
    import inspect
    src = inspect.getsource(bench.main)
    assert 'default="fusion"' in src
    assert bench.WORKLOADS["fusion"]["precision"] == "ref"   # the headline is at reference numerics
    assert bench.WORKLOADS["stress4"]["precision"] == "fp16"


def test_flop_accounting_matches_survey():
    # 245.0 / 415.5 / 603.6 / 2210 GFLOP per decoder-frame
    assert abs(bench.decoder_frame_flops() / 1e9 - 245.0) < 0.1
    assert abs(bench.decoder_frame_flops(nk=56400) / 1e9 - 415.5) < 0.1
    coop = bench.decoder_frame_flops(nk=36400) + bench.decoder_frame_flops(nk=44400)
    assert abs(coop / 1e9 - 603.6) < 0.1
    stress = 4 * bench.decoder_frame_flops(nq=1500, nk=48400)
    assert abs(stress / 1e9 - 2210) < 5
    assert bench.cross_attn_flops() == 4.0 * 900 * 32400 * 256


def test_headline_traffic_profile_committed():
    traffic, src = bench.load_traffic("fusion", 56400)
    assert traffic > 0 and src.startswith("profiles/")


def test_missing_traffic_profile_fails_loudly():
    import pytest
    with pytest.raises(RuntimeError):
        bench.load_traffic("fusion", 12345)


def test_cpu_threads_respects_omp(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert 1 <= bench.cpu_threads() <= 3


def test_bench_line_names_what_it_keeps():
    """The headline keeps weight-only encodings like weight packs: the line must
    list each of them and carry the recomputed-per-frame side key."""
    import inspect
    src = inspect.getsource(bench.main)
    assert '"weight_only_kept"' in src and '"weight_only_recomputed"' in src
    assert len(bench.WEIGHT_ONLY_KEPT) == 3
    assert "with_metas(head, metas, run" in src     # every timed step re-stages the camera matrices ...
    assert "stage_metas" in inspect.getsource(bench.with_metas)   # ... (host fp64 inverse + staging)
    # every other BASELINE config's number rides on the default line
    assert all(k in src for k in ('"lidar"', '"stress4"', '"train_coop"'))
    _, _, fwd, _, _ = bench.make_workload("fusion", seed=0)
    assert len(fwd.metas) == 1 and "lidar2img" in fwd.metas[0]
