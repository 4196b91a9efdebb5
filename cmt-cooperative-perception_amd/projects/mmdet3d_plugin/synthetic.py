"""Synthetic frames, camera geometry and seeded weights for the BASELINE.json
configs (no datasets or checkpoints are available offline).

  * BEV features  [B, 512, H, W] = relu(N(0,1))  (SECONDFPN ends in BN+ReLU)
  * image features [B*V, 256, 40, 100] ~ N(0,1)  (CPFPN output, 1600x640 / 16)
  * lidar2img: f = 1266, principal point (800, 190) (900-row image bottom-cropped
    to 640, transform_3d.py:449-457), cameras 1.5 m above the LiDAR origin at the
    given yaws; pad_shape (640, 1600, 3)
  * points [N, 5]: xyz uniform in the point-cloud range, intensity U[0,255],
    time-lag U[0, 0.5]
  * weights: the reference's init (xavier decoder, kaiming task heads, cls bias
    -2.19, reference_points U(0,1)), optionally with biases / norm affine
    parameters jittered so every fused epilogue is exercised by the parity tests.
"""
import copy
import math
import os

import numpy as np
import torch

from .config import load_config
from .registry import build_head

__all__ = ["CONFIG_DIR", "make_head_cfg", "build_synthetic_head", "camera_lidar2img", "synthetic_metas",
           "synthetic_bev", "synthetic_img", "synthetic_points", "head_state_dict", "CONFIGS"]

CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs")
CONFIGS = ("cmt_lidar_nus", "cmt_fusion_nus", "cmtcoop_fusion_tumtraf", "cmtcoop_lidar_tumtraf")

NUS_YAWS = (0.0, 55.0, -55.0, 110.0, -110.0, 180.0)
VEHICLE_YAWS = (0.0,)
INFRA_YAWS = (30.0, 150.0, -90.0)


def make_head_cfg(name, num_query=900, num_layers=None, grid_size=None, head_type=None):
    """The ``pts_bbox_head`` dict of a reference config (plus train/test cfg)."""
    base = load_config(os.path.join(CONFIG_DIR, "_decoder.py"))
    c = load_config(os.path.join(CONFIG_DIR, name + ".py"))
    decoder = copy.deepcopy(base["decoder"])
    if num_layers is not None:
        decoder["num_layers"] = num_layers
    classes = c.get("nus_classes") or c.get("tumtraf_classes")
    grid = list(grid_size) if grid_size is not None else list(c["grid_size"])
    head = dict(
        type=head_type or c["head_type"], in_channels=512, hidden_dim=256, downsample_scale=8, num_query=num_query,
        common_heads=copy.deepcopy(base["common_heads"]),
        tasks=[dict(num_class=len(classes), class_names=list(classes))],
        bbox_coder=dict(type="MultiTaskBBoxCoder", post_center_range=c["post_center_range"],
                        pc_range=c["point_cloud_range"], max_num=300, voxel_size=c["voxel_size"],
                        num_classes=len(classes)),
        separate_head=dict(type="SeparateTaskHead", init_bias=-2.19, final_kernel=c["final_kernel"]),
        transformer=dict(type=c["transformer_type"], decoder=decoder),
        # the reference configs' losses (e.g. CMTCoop_TUMTraf/fusion/coop/...py:327-328)
        loss_cls=dict(type="FocalLoss", use_sigmoid=True, gamma=2, alpha=0.25, reduction="mean", loss_weight=2.0),
        loss_bbox=dict(type="L1Loss", reduction="mean", loss_weight=0.25),
        train_cfg=None,
        test_cfg=dict(grid_size=grid, out_size_factor=8, pc_range=c["point_cloud_range"], voxel_size=c["voxel_size"],
                      nms_type=None, max_num=200),
    )
    return head, c


def _jitter_(module, gen, scale=0.05):
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith("bias") or ("norm" in name and name.endswith("weight")) or ".1.weight" in name:
                p.add_(torch.randn(p.shape, generator=gen) * scale)
        for name, b in module.named_buffers():
            if name.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=gen) * 0.1)
            elif name.endswith("running_var"):
                b.copy_(torch.rand(b.shape, generator=gen) * 0.5 + 0.75)


def build_synthetic_head(name, *, seed=0, num_query=900, num_layers=None, grid_size=None, jitter=True,
                         device=None):
    cfg, meta = make_head_cfg(name, num_query=num_query, num_layers=num_layers, grid_size=grid_size)
    torch.manual_seed(seed)
    head = build_head(cfg)
    head.init_weights()
    if jitter:
        _jitter_(head, torch.Generator().manual_seed(seed + 1))
    head.eval()
    if device is not None:
        head.to(device)
    return head, cfg, meta


def head_state_dict(head):
    return {k: v.detach().float().cpu() for k, v in head.state_dict().items()}


def camera_lidar2img(yaw_deg, height=1.5, f=1266.0, cx=800.0, cy=190.0):
    """4x4 lidar->image projection of a pinhole camera at (0, 0, height)
    looking along yaw (x right, y down, z forward in the camera frame)."""
    t = math.radians(yaw_deg)
    fwd = np.array([math.cos(t), math.sin(t), 0.0])
    right = np.array([math.sin(t), -math.cos(t), 0.0])
    down = np.array([0.0, 0.0, -1.0])
    R = np.stack([right, down, fwd])
    c = np.array([0.0, 0.0, height])
    E = np.eye(4)
    E[:3, :3] = R
    E[:3, 3] = -R @ c
    K = np.eye(4)
    K[0, 0] = K[1, 1] = f
    K[0, 2], K[1, 2] = cx, cy
    return K @ E


def synthetic_metas(B, yaws=NUS_YAWS, pad_shape=(640, 1600, 3), prefix="", seed=0, extra=None):
    """img_metas with ``lidar2img`` (intrinsics scaled to pad_shape from the
    1600x640 nuScenes crop) and ``pad_shape``; ``prefix`` = '' / 'vehicle_' /
    'infrastructure_' (the coop meta convention, cmt_head_coop.py:41-69)."""
    rng = np.random.default_rng(seed)
    sx, sy = pad_shape[1] / 1600.0, pad_shape[0] / 640.0
    metas = []
    for _ in range(B):
        # small per-frame extrinsic jitter so batch entries differ
        l2i = [camera_lidar2img(y + rng.uniform(-2, 2), height=1.5 + rng.uniform(-0.1, 0.1), f=1266.0 * sx,
                                cx=800.0 * sx, cy=190.0 * sy) for y in yaws]
        m = {prefix + "lidar2img": l2i, prefix + "pad_shape": [pad_shape] * len(yaws)}
        metas.append(m)
    if extra is not None:
        for m, e in zip(metas, extra):
            m.update(e)
    return metas


def synthetic_bev(B, H=180, W=180, C=512, seed=0, device=None):
    g = torch.Generator().manual_seed(seed)
    x = torch.relu(torch.randn((B, C, H, W), generator=g))
    return x.to(device) if device is not None else x


def synthetic_img(BV, h=40, w=100, C=256, seed=0, device=None):
    g = torch.Generator().manual_seed(seed + 7)
    x = torch.randn((BV, C, h, w), generator=g)
    return x.to(device) if device is not None else x


def synthetic_gt(B, pc_range, num_classes, n=20, seed=0, device=None):
    """Training targets (20 boxes per frame):
    gravity-centre boxes [n, 9] (x, y, z, w, l, h, yaw, vx, vy) inside the
    central 70 % of the range, dims 1-4 m, and labels < num_classes."""
    g = torch.Generator().manual_seed(seed + 29)
    boxes, labels = [], []
    lo, hi = torch.tensor(pc_range[:3]), torch.tensor(pc_range[3:])
    for _ in range(B):
        c = lo + (hi - lo) * (0.15 + 0.7 * torch.rand(n, 3, generator=g))
        d = 1.0 + 3.0 * torch.rand(n, 3, generator=g)
        yaw = (torch.rand(n, 1, generator=g) * 2 - 1) * math.pi
        vel = torch.randn(n, 2, generator=g)
        b = torch.cat([c, d, yaw, vel], 1)
        l = torch.randint(0, num_classes, (n,), generator=g)
        boxes.append(b.to(device) if device is not None else b)
        labels.append(l.to(device) if device is not None else l)
    return boxes, labels


def synthetic_points(N, pc_range, seed=0, device=None, margin=0.0):
    g = torch.Generator().manual_seed(seed + 13)
    lo = torch.tensor(pc_range[:3], dtype=torch.float32) - margin
    hi = torch.tensor(pc_range[3:], dtype=torch.float32) + margin
    xyz = lo + torch.rand((N, 3), generator=g) * (hi - lo)
    inten = torch.rand((N, 1), generator=g) * 255.0
    dt = torch.rand((N, 1), generator=g) * 0.5
    p = torch.cat([xyz, inten, dt], 1)
    return p.to(device) if device is not None else p
