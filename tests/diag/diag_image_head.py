"""Diagnostic: image-only head parity -- compares the rv query geometry
(coords + view mask) of the native kernel with the oracle's einsum path and
reports where the head outputs differ most."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import cmt_oracle as O  # noqa: E402
from projects.mmdet3d_plugin import build_head, native, set_precision  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402

dev = torch.device("cuda:0")
cfg, _ = S.make_head_cfg("cmt_fusion_nus", num_query=40, num_layers=2, grid_size=[256, 256, 40],
                         head_type="CmtImageHead")
cfg["transformer"]["type"] = "CmtImageTransformer"
torch.manual_seed(0)
head = build_head(cfg)
head.init_weights()
head.eval()
sd = S.head_state_dict(head)
oc = O.cfg_from_head_cfg(cfg)
B, cams = 2, 3
xi = S.synthetic_img(B * cams, 8, 20, seed=5)
metas = S.synthetic_metas(B, yaws=S.NUS_YAWS[:cams], pad_shape=(128, 320, 3), seed=6)
ref = O.head_forward(oc, sd, None, xi, metas, "image", cross_core="fp16", self_core="fp32")[0]
head.to(dev)
set_precision("ref")
with torch.no_grad():
    got = head([None], [xi.to(dev)], metas)[0][0]
for k in ("cls_logits", "dim", "rot", "vel", "center", "height"):
    e = (got[k].cpu() - ref[k]).abs()
    idx = np.unravel_index(int(e.argmax()), e.shape)
    print(k, "max", f"{e.max().item():.3e}", "at", idx, "mean", f"{e.mean().item():.2e}")
# geometry: GPU kernel vs oracle's mask
ref_pts = sd["reference_points.weight"]
Nq = ref_pts.shape[0]
l2i = np.stack([np.asarray(m["lidar2img"], np.float64) for m in metas])
i2l = np.linalg.inv(l2i)
coords = torch.empty(B * cams * Nq, 192, device=dev)
mask = torch.empty(B * cams * Nq, device=dev)
native.rv_query_coords(ref_pts.unsqueeze(0).expand(B, Nq, 3).contiguous().to(dev),
                       torch.from_numpy(l2i).float().to(dev), torch.from_numpy(i2l).float().to(dev), coords, mask,
                       B=B, V=cams, Nq=Nq, D=64, pad_h=128.0, pad_w=320.0, pc_range=oc["pc_range"])
# oracle geometry (replicates rv_query_embed up to the mask)
pcr = torch.tensor(oc["pc_range"])
rp = O.inverse_sigmoid(ref_pts.unsqueeze(0).repeat(B, 1, 1)).sigmoid()
rp = rp * (pcr[3:] - pcr[:3]) + pcr[:3]
proj = torch.einsum("bnd, bvcd -> bvnc", torch.cat([rp, torch.ones(B, Nq, 1)], -1), torch.from_numpy(l2i).float())
z = proj[..., 2:3]
zm = z > 0
pp = proj[..., :3] / (z + zm * 1e-6 - (~zm) * 1e-6)
m = (pp[..., 0] < 320) & (pp[..., 0] >= 0) & (pp[..., 1] < 128) & (pp[..., 1] >= 0) & zm.squeeze(-1)
gm = mask.view(B, cams, Nq).cpu().bool()
print("mask flips:", int((gm != m).sum()), "of", m.numel(), "; visible:", int(m.sum()))
print("min |x - border| over visible:", float(torch.stack([pp[..., 0], 320 - pp[..., 0], pp[..., 1], 128 - pp[..., 1]]).abs().min()))
