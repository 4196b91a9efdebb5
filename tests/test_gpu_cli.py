"""BASELINE.json configs[0] through the tools/test.py-shaped CLI on the GPU:
CMT-L head, 1 decoder layer, 32 queries, 1 000 points uniform in the
point-cloud range (seed 0), --synthetic, in this process.  Checks that the
CLI's boxes equal a direct head forward + get_bboxes on the same inputs, that
its voxel counts equal the C oracle voxelizer's on the same points (bit-exact
integer work), and that --format-only writes OpenLABEL files whose point
counts match the closed-form point-in-box test."""
import ctypes
import importlib.util
import json
import os

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

ARGS = ["cmt_lidar_nus", "--synthetic", "--num-query", "32", "--num-layers", "1", "--points", "1000",
        "--grid", "180", "180", "--seed", "0"]


def _cli():
    spec = importlib.util.spec_from_file_location("cmt_test_cli", os.path.join(PKG, "tools", "test.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _oracle_voxel_count(points, layer_cfg):
    lib_path = os.path.join(ROOT, "oracle", "_build", "libvoxel_oracle.so")
    if not os.path.exists(lib_path):
        pytest.skip("oracle voxelizer not built (build() compiles it)")
    lib = ctypes.CDLL(lib_path)
    fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    pts = np.ascontiguousarray(points, np.float32)
    N, F = pts.shape
    mv = layer_cfg["max_voxels"][1]
    mp = layer_cfg["max_num_points"]
    rng = np.array(layer_cfg["point_cloud_range"], np.float32)
    vs = np.array(layer_cfg["voxel_size"], np.float32)
    grid = np.round((rng[3:] - rng[:3]) / vs).astype(np.int32)
    v = np.zeros((mv, mp, F), np.float32)
    c = np.zeros((mv, 3), np.int32)
    n = np.zeros((mv,), np.int32)
    m = np.zeros((mv, F), np.float32)
    M = lib.cmt_oracle_voxelize(pts.ctypes.data_as(fp), N, F, vs.ctypes.data_as(fp), rng.ctypes.data_as(fp),
                                grid.ctypes.data_as(ip), mp, mv, F, v.ctypes.data_as(fp), c.ctypes.data_as(ip),
                                n.ctypes.data_as(ip), m.ctypes.data_as(fp))
    return int(M), int(n[:M].sum())


def _direct(cli, head, feats, metas, precision):
    from projects.mmdet3d_plugin import get_precision, set_precision
    prev = get_precision()
    set_precision(precision)
    try:
        with torch.no_grad():
            return cli.run_frame(head, "cmt_lidar_nus", feats, metas)
    finally:
        set_precision(prev)


def test_config1_cli_matches_direct_forward(dev, tmp_path, parity_log):
    cli = _cli()
    out = tmp_path / "r.json"
    assert cli.main(ARGS + ["--out", str(out), "--eval", "bbox"]) == 0
    res = json.load(open(out))
    assert res["config"] == "cmt_lidar_nus" and len(res["frames"]) == 1
    fr = res["frames"][0]

    # the same frame directly through the head, under the CLI's compute policy
    args = cli.parse_args(ARGS + ["--eval", "bbox"])
    head, cfg, meta = cli.build_head(args, "cmt_lidar_nus", dev)
    feats, metas, points = cli.frame_inputs("cmt_lidar_nus", meta, 0, args, dev)
    boxes, scores, labels = _direct(cli, head, feats, metas, args.precision)
    assert fr["labels_3d"] == labels.cpu().tolist()
    np.testing.assert_array_equal(np.asarray(fr["scores_3d"], np.float32), scores.float().cpu().numpy())
    np.testing.assert_array_equal(np.asarray(fr["boxes_3d"], np.float32).reshape(-1, 9),
                                  boxes.float().cpu().numpy())
    assert len(fr["scores_3d"]) > 0

    # voxel layer vs the C oracle on the same 1 000 points
    M, kept = _oracle_voxel_count(points[0].cpu().numpy(), dict(meta["pts_voxel_layer"]))
    assert fr["voxels"][0] == {"voxels": M, "points_kept": kept}
    parity_log.append(f"configs[0] CLI (CMT-L, L 1, Nq 32, 1000 points): {len(fr['scores_3d'])} boxes, "
                      f"voxels {M} / points kept {kept} == oracle, CLI == direct forward bit-exact")


def test_config1_cli_openlabel(dev, tmp_path):
    from projects.mmdet3d_plugin.core.openlabel import points_in_box
    cli = _cli()
    od = tmp_path / "ol"
    assert cli.main(ARGS + ["--frames", "2", "--format-only", "--openlabel-dir", str(od), "--bbox-score",
                            "0.0"]) == 0
    files = sorted(os.listdir(od))
    assert files == ["frame_000000.json", "frame_000001.json"]
    args = cli.parse_args(ARGS + ["--format-only"])
    head, cfg, meta = cli.build_head(args, "cmt_lidar_nus", dev)
    for f, name in enumerate(files):
        ol = json.load(open(od / name))["openlabel"]
        objs = ol["frames"][str(f)]["objects"]
        feats, metas, points = cli.frame_inputs("cmt_lidar_nus", meta, f, args, dev)
        boxes, scores, labels = _direct(cli, head, feats, metas, args.precision)
        assert len(objs) == len(scores)
        pts = points[0][:, :3].cpu().numpy()
        got = sorted(o["object_data"]["cuboid"]["attributes"]["num"][0]["val"] for o in objs.values())
        b = boxes.float().cpu().numpy()
        want = sorted(points_in_box(pts, bx[:3], bx[3:6], float(bx[6])) for bx in b)
        assert got == want
