"""Checkpoint formats: the head's mmcv key layout and the
CmtDetector -> CmtCoopDetector key rewrite of
tools/model_converters/convert_cmtcoop_checkpoints.py (restated in
projects/mmdet3d_plugin/checkpoint.py; the reference script needs mmcv/mmdet3d
and a built detector, so parity is on its rules: delete, insert prefix,
permute, merge order)."""
import torch

from projects.mmdet3d_plugin import synthetic as S
from projects.mmdet3d_plugin.checkpoint import (convert_agent_checkpoint, load_head_checkpoint,
                                                merge_coop_checkpoints)


def _detector_sd(head, seed):
    g = torch.Generator().manual_seed(seed)
    sd = {"pts_bbox_head." + k: v.clone() for k, v in head.state_dict().items()}
    sd["pts_backbone.blocks.0.0.weight"] = torch.randn(4, 3, 3, 3, generator=g)
    sd["pts_middle_encoder.conv_input.0.weight"] = torch.randn(16, 3, 3, 3, 5, generator=g)   # spconv v1 layout
    sd["pts_middle_encoder.conv_input.1.weight"] = torch.randn(16, generator=g)               # BN: not permuted
    sd["img_backbone.stem.weight"] = torch.randn(8, 3, 3, 3, generator=g)
    return sd


def test_head_checkpoint_roundtrip(tmp_path):
    head, _, _ = S.build_synthetic_head("cmt_lidar_nus", num_query=16, num_layers=1, grid_size=[256, 256, 40])
    p = tmp_path / "det.pth"
    torch.save({"state_dict": _detector_sd(head, 0), "meta": {"epoch": 1}}, p)
    other, _, _ = S.build_synthetic_head("cmt_lidar_nus", seed=5, num_query=16, num_layers=1,
                                         grid_size=[256, 256, 40])
    missing, unexpected = load_head_checkpoint(other, str(p))
    assert not missing and not unexpected
    for k, v in head.state_dict().items():
        assert torch.equal(other.state_dict()[k], v), k


def test_agent_conversion_rules():
    head, _, _ = S.build_synthetic_head("cmt_lidar_nus", num_query=16, num_layers=1, grid_size=[256, 256, 40])
    sd = _detector_sd(head, 1)
    sd["infrastructure_model.pts_neck.w"] = torch.zeros(1)
    out = convert_agent_checkpoint(sd, "vehicle")
    assert not any(k.startswith("pts_bbox_head.task_heads") for k in out)          # DEL_PREFIX
    assert not any(k.startswith("infrastructure_model") for k in out)              # the other agent's extractor
    assert "vehicle_model.pts_backbone.blocks.0.0.weight" in out                    # INSERT_PREFIX
    assert "vehicle_model.img_backbone.stem.weight" in out
    w = out["vehicle_model.pts_middle_encoder.conv_input.0.weight"]
    assert w.shape == (3, 3, 3, 5, 16)                                              # PERMUTE (1, 2, 3, 4, 0)
    assert torch.equal(w, sd["pts_middle_encoder.conv_input.0.weight"].permute(1, 2, 3, 4, 0))
    assert out["vehicle_model.pts_middle_encoder.conv_input.1.weight"].shape == (16,)
    assert "pts_bbox_head.transformer.decoder.post_norm.weight" in out
    assert "pts_bbox_head.transformer.decoder.post_norm.weight" not in convert_agent_checkpoint(sd, "vehicle",
                                                                                                wo_trans=True)
    lidar_only = convert_agent_checkpoint(sd, "vehicle", prefix="pts")
    assert "img_backbone.stem.weight" in lidar_only                                 # not renamed for prefix 'pts'


def test_coop_merge_and_head_load():
    hv, _, _ = S.build_synthetic_head("cmt_lidar_nus", seed=1, num_query=16, num_layers=1, grid_size=[256, 256, 40])
    hi, _, _ = S.build_synthetic_head("cmt_lidar_nus", seed=2, num_query=16, num_layers=1, grid_size=[256, 256, 40])
    merged = merge_coop_checkpoints(vehicle=_detector_sd(hv, 3), infrastructure=_detector_sd(hi, 4))
    assert "vehicle_model.pts_backbone.blocks.0.0.weight" in merged
    assert "infrastructure_model.pts_backbone.blocks.0.0.weight" in merged
    # shared head keys: the infrastructure checkpoint is merged last and wins (main: {**vehicle, **infra})
    k = "pts_bbox_head.shared_conv.conv.weight"
    assert torch.equal(merged[k], hi.state_dict()["shared_conv.conv.weight"])
    coop, _, _ = S.build_synthetic_head("cmtcoop_lidar_tumtraf", num_query=16, num_layers=1,
                                        grid_size=[256, 256, 40])
    missing, unexpected = load_head_checkpoint(coop, merged, strict=False)
    assert not unexpected
    assert missing and all(m.startswith("task_heads") for m in missing)   # re-initialised, as in the reference
