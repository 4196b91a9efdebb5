"""bench.py host logic on CPU: the three workloads build with the shapes
BASELINE.json names, and the FLOP accounting matches the
survey's per-frame figures."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_workload_shapes():
    expect = {"lidar": ([32400], "CmtLidarHead"), "fusion": ([56400], "CmtHead"),
              "coop": ([36400, 44400], "CmtHeadCoop")}
    for name, (nks, cls) in expect.items():
        head, cfg, fwd, got, oracle_fwd = bench.make_workload(name, seed=0)
        assert got == nks, name
        assert type(head).__name__ == cls
        assert head.num_query == 900 and head.transformer.decoder.num_layers == 6
        assert callable(fwd) and callable(oracle_fwd)


def test_flop_accounting_matches_survey():
    # 245.0 / 415.5 / 603.6 GFLOP per decoder-frame
    assert abs(bench.decoder_frame_flops() / 1e9 - 245.0) < 0.1
    assert abs(bench.decoder_frame_flops(nk=56400) / 1e9 - 415.5) < 0.1
    coop = bench.decoder_frame_flops(nk=36400) + bench.decoder_frame_flops(nk=44400)
    assert abs(coop / 1e9 - 603.6) < 0.1
    assert bench.cross_attn_flops() == 4.0 * 900 * 32400 * 256
