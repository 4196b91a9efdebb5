"""OpenLABEL export (core/openlabel.py, after inference_to_openlabel_coop.py) and
the tools/test.py-shaped CLI's host side: argument contract, --cfg-options,
and the loud failure without a HIP device (no CPU path)."""
import importlib.util
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT


def _cli():
    spec = importlib.util.spec_from_file_location("cmt_test_cli", os.path.join(PKG, "tools", "test.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_box_corners_kat():
    from projects.mmdet3d_plugin.core.openlabel import box_corners
    c = box_corners(math.pi / 2, width=2.0, length=4.0, position=np.array([1.0, 2.0, 3.0]))
    # heading +y: +-2 along y, +-1 along -x
    np.testing.assert_allclose(c, [[0.0, 4.0, 3.0], [0.0, 0.0, 3.0], [2.0, 0.0, 3.0], [2.0, 4.0, 3.0]], atol=1e-12)


def test_openlabel_json_structure(tmp_path):
    from projects.mmdet3d_plugin.core.openlabel import Detection, detections_to_openlabel
    d = Detection(location=np.array([[1.0], [2.0], [3.5]]), dimensions=(4.0, 2.0, 1.5), yaw=math.pi / 2,
                  category="car", uuid="abcd-ef", num_lidar_points=7, score=0.875, sensor_id="s110")
    out = detections_to_openlabel([d], filename="f.json", output_folder_path=str(tmp_path), frame_id=3)
    with open(tmp_path / "f.json") as f:
        assert json.load(f) == json.loads(json.dumps(out))
    ol = out["openlabel"]
    assert ol["metadata"] == {"schema_version": "1.0.0"} and ol["coordinate_systems"] == {}
    obj = ol["frames"]["3"]["objects"]["abcd-ef"]["object_data"]
    assert obj["name"] == "CAR_abcd" and obj["type"] == "CAR" and obj["bbox"] == []
    val = obj["cuboid"]["val"]
    s = math.sqrt(0.5)
    np.testing.assert_allclose(val, [1.0, 2.0, 3.5, 0.0, 0.0, s, s, 4.0, 2.0, 1.5], atol=1e-12)
    attrs = obj["cuboid"]["attributes"]
    assert attrs["text"] == [{"name": "overlap", "val": "False"}, {"name": "sensor_id", "val": "s110"}]
    assert attrs["num"] == [{"name": "num_points", "val": 7}, {"name": "score", "val": 0.875}]
    assert attrs["vec"] == [{"name": "track_history", "val": []}]


def test_openlabel_optional_fields():
    from projects.mmdet3d_plugin.core.openlabel import Detection, detections_to_openlabel
    d = Detection(location=np.zeros(3), dimensions=(1, 1, 1), yaw=0.0, category="van", uuid="", color="Red",
                  occlusion_level="PARTIALLY", bbox_2d=np.array([10.0, 20.0, 30.0, 60.0]),
                  pos_history=[np.array([1.0, 2.0, 3.0]), np.array([4.0, 5.0, 6.0])])
    out = detections_to_openlabel([d], frame_properties={"t": 1}, streams={"s": {}},
                                  coordinate_systems={"lidar": {}})
    ol = out["openlabel"]
    obj = ol["frames"]["0"]["objects"]["0"]["object_data"]          # empty uuid -> the list index
    assert obj["bbox"] == [{"name": "shape", "val": [20.0, 40.0, 20.0, 40.0]}]
    text = [a["name"] for a in obj["cuboid"]["attributes"]["text"]]
    assert text == ["body_color", "overlap", "occlusion_level", "sensor_id"]
    assert obj["cuboid"]["attributes"]["text"][0]["val"] == "red"
    assert obj["cuboid"]["attributes"]["vec"][0]["val"] == [1.0, 2.0, 3.0, 4.0, 5.0, 6.0]
    assert ol["frames"]["0"]["frame_properties"] == {"t": 1} and ol["streams"] == {"s": {}}
    assert ol["coordinate_systems"] == {"lidar": {}}


def test_boxes_to_detections_filters_and_point_count():
    from projects.mmdet3d_plugin.core.openlabel import boxes_to_detections, points_in_box
    # x, y, z_bottom, dx, dy, dz, yaw, vx, vy
    boxes = np.array([[0.0, 0.0, 0.0, 4.0, 2.0, 2.0, math.pi / 2, 0, 0],
                      [10.0, 0.0, 0.0, 1.0, 1.0, 1.0, 0.0, 0, 0],
                      [20.0, 0.0, 0.0, 1.0, 1.0, 1.0, 0.0, 0, 0]])
    scores = np.array([0.9, 0.2, 0.6])
    labels = np.array([0, 1, 2])
    # the box is rotated 90 deg: extent 4 along y, 2 along x; centred at (0, 0, 0) (the bottom centre, as the
    # reference's open3d box) so z in [-1, 1] counts
    pts = np.array([[0.0, 1.9, 0.5], [0.0, 2.1, 0.0], [0.9, 0.0, -0.9], [1.1, 0.0, 0.0], [0.0, 0.0, 1.2]])
    assert points_in_box(pts, boxes[0, :3], boxes[0, 3:6], boxes[0, 6]) == 2
    ids = iter(["u0", "u1", "u2"])
    dets = boxes_to_detections(boxes, scores, labels, ["car", "van", "bus"], points_xyz=pts, bbox_score=0.5,
                               uuid_fn=lambda: next(ids))
    assert [d.category for d in dets] == ["car", "bus"]
    assert dets[0].num_lidar_points == 2 and dets[1].num_lidar_points == 0
    np.testing.assert_allclose(dets[0].location.flatten(), [0.0, 0.0, 1.0])   # z lifted by h / 2
    assert dets[0].yaw == -math.pi / 2 and dets[0].dimensions == (4.0, 2.0, 2.0)
    assert [d.uuid for d in dets] == ["u0", "u1"]
    only_van = boxes_to_detections(boxes, scores, labels, ["car", "van", "bus"], bbox_classes=[1])
    assert len(only_van) == 1 and only_van[0].category == "van" and only_van[0].num_lidar_points == 0


def test_cli_argument_contract():
    cli = _cli()
    with pytest.raises(SystemExit):
        cli.parse_args(["cmt_lidar_nus", "--synthetic"])                      # no operation
    with pytest.raises(SystemExit):
        cli.parse_args(["cmt_lidar_nus", "--synthetic", "--eval", "bbox", "--format-only"])
    with pytest.raises(SystemExit):
        cli.parse_args(["cmt_lidar_nus", "--eval", "bbox"])                   # datasets out of scope
    with pytest.raises(SystemExit):
        cli.parse_args(["cmt_lidar_nus", "--synthetic", "--out", "r.pkl"])   # JSON results
    a = cli.parse_args(["projects/configs/cmt_lidar_nus.py", "--synthetic", "--num-query", "32", "--num-layers",
                        "1", "--points", "1000", "--eval", "bbox", "--cfg-options", "test_cfg.max_num=50",
                        "bbox_coder.score_threshold=0.1"])
    assert cli.config_name(a.config) == "cmt_lidar_nus"
    with pytest.raises(SystemExit):
        cli.config_name("foo.py")
    cfg = cli.apply_cfg_options({"test_cfg": {"max_num": 200}, "bbox_coder": {}}, a.cfg_options)
    assert cfg["test_cfg"]["max_num"] == 50 and cfg["bbox_coder"]["score_threshold"] == 0.1


def test_cli_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present (the GPU test runs the CLI)")
    r = subprocess.run([sys.executable, os.path.join(PKG, "tools", "test.py"), "cmt_lidar_nus", "--synthetic",
                        "--num-query", "32", "--num-layers", "1", "--eval", "bbox"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "no HIP device" in r.stderr, (r.returncode, r.stderr[-500:])
