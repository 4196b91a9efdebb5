"""Merge single-agent CMT checkpoints into one CMTCoop checkpoint (the CLI of
the reference's tools/model_converters/convert_cmtcoop_checkpoints.py:20-33,
287-372, without building the detector; key rules in
projects/mmdet3d_plugin/checkpoint.py).

    python cmt-cooperative-perception_amd/tools/convert_cmtcoop_checkpoints.py \
        --vehicle_checkpoint v.pth --infrastructure_checkpoint i.pth --out coop.pth
    (or --vehicle_lidar / --vehicle_camera / --infrastructure_lidar / --infrastructure_camera)

With ``--config`` the merged head keys are also loaded into a freshly built
head of that config (strict=False, as the reference's check).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from projects.mmdet3d_plugin.checkpoint import load_head_checkpoint, merge_coop_checkpoints  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description="Convert CmtDetector checkpoints to a CmtCoopDetector checkpoint")
    ap.add_argument("--config", help="synthetic head config name (projects/configs) to check the head keys against")
    for a in ("vehicle_checkpoint", "infrastructure_checkpoint", "vehicle_lidar", "vehicle_camera",
              "infrastructure_lidar", "infrastructure_camera"):
        ap.add_argument("--" + a)
    ap.add_argument("--wo_trans", action="store_true", help="drop pts_bbox_head.transformer as well")
    ap.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    sd = merge_coop_checkpoints(vehicle=args.vehicle_checkpoint, infrastructure=args.infrastructure_checkpoint,
                                vehicle_lidar=args.vehicle_lidar, vehicle_camera=args.vehicle_camera,
                                infrastructure_lidar=args.infrastructure_lidar,
                                infrastructure_camera=args.infrastructure_camera, wo_trans=args.wo_trans)
    if args.config:
        from projects.mmdet3d_plugin import synthetic as S
        head, _, _ = S.build_synthetic_head(args.config, jitter=False)
        missing, unexpected = load_head_checkpoint(head, sd, strict=False)
        print(f"head check: {len(missing)} missing, {len(unexpected)} unexpected keys")
    d = os.path.dirname(args.out)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save(sd, args.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
