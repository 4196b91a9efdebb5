"""Diagnostics: where the 'ref' policy's logit error vs the fp16-core oracle
comes from (configs[2] fusion, full size): split vs exact GEMMs x bounded vs
online f16 cross-attention offsets."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cmt-cooperative-perception_amd")]
import torch  # noqa: E402

from oracle import cmt_oracle as O  # noqa: E402
from projects.mmdet3d_plugin import native, set_precision  # noqa: E402
from projects.mmdet3d_plugin import synthetic as S  # noqa: E402

KEYS = ("center", "height", "dim", "rot", "vel", "cls_logits")
dev = torch.device("cuda:0")
head, cfg, _ = S.build_synthetic_head("cmt_fusion_nus", seed=0, num_query=900)
oc, sd = O.cfg_from_head_cfg(cfg), S.head_state_dict(head)
x = S.synthetic_bev(1, 180, 180, seed=42)
xi = S.synthetic_img(6, 40, 100, seed=43)
metas = S.synthetic_metas(1, yaws=S.NUS_YAWS, seed=44)
ref = O.head_forward(oc, sd, x, xi, metas, "fusion", cross_core="fp16", epilogue=False)[0]
ref32 = O.head_forward(oc, sd, x, xi, metas, "fusion", cross_core="fp32", epilogue=False)[0]
head.to(dev)
head.box_epilogue = False
xd, xid = x.to(dev), xi.to(dev)
orig_attn = native.attention


def no_bound(*a, **k):
    k["kmax2"] = None
    k["kmax_ld"] = 0
    return orig_attn(*a, **k)


def err(got, r):
    return max((got[k].detach().cpu().double() - r[k].double()).abs().max().item() for k in KEYS)


print(f"oracle fp16 core vs oracle fp32 core: {err({k: ref[k] for k in KEYS}, ref32):.2e}", flush=True)
for prec in ("ref", "exact"):
    for mode in ("bounded", "online"):
        native.attention = orig_attn if mode == "bounded" else no_bound
        set_precision(prec)
        with torch.no_grad():
            got = head([xd], [xid], metas)[0][0]
        torch.cuda.synchronize()
        print(f"{prec:6s} {mode:8s}: max abs vs fp16-core oracle {err(got, ref):.2e}  "
              f"(vs fp32-core oracle {err(got, ref32):.2e})", flush=True)
native.attention = orig_attn
