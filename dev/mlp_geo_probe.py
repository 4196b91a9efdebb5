"""Times the camera memory rows at the fusion frame's shape (6 x 40 x 100 tokens, depth_num 64):
the one-launch form (cmt_mlp2_x3 with geo + rx, ABI 20) against coordinates kernel + layout pass +
one-launch MLP.  HIP events, mean of 20 launches after 3 warm-ups.
    python dev/mlp_geo_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmt-cooperative-perception_amd"))
from projects.mmdet3d_plugin import native  # noqa: E402

dev = torch.device("cuda:0")
B, V, h, w, D, C, Hd = 1, 6, 40, 100, 64, 256, 1024
M = V * h * w
Nk = 32400 + M
g = torch.Generator().manual_seed(0)
W1 = torch.randn(Hd, 3 * D, generator=g) / 14
W2 = torch.randn(C, Hd, generator=g) / 32


def pair(x):
    hi = x.half()
    return torch.stack([hi, (x - hi.float()).half()], dim=-2).contiguous().view(torch.uint16)


W1p, W2p = native.mlp2_pack(pair(W1).to(dev), pair(W2).to(dev))
b1 = (torch.randn(Hd, generator=g) / 10).to(dev)
b2 = (torch.randn(C, generator=g) / 10).to(dev)
i2l = torch.eye(4).repeat(B, V, 1, 1) + 0.01 * torch.randn(B, V, 4, 4, generator=g)
i2l = i2l.to(dev).contiguous()
xi = torch.randn(B * V, C, h, w, generator=g).to(dev)
mem = torch.empty((B * Nk, 2, C), dtype=torch.uint16, device=dev)
pos = torch.empty((B * Nk, 2, C), dtype=torch.uint16, device=dev)
pc = [-54.0, -54.0, -5.0, 54.0, 54.0, 3.0]
geo = dict(i2l=i2l, h=h, w=w, D=D, pad_h=640.0, pad_w=1600.0, depth_max=54.0, pc_range=pc)
coords = torch.empty((B * M, 2, 3 * D), dtype=torch.uint16, device=dev)


def fused():
    native.mlp2(None, W1p, b1, W2p, b2, pos, M=M, K=3 * D, Hd=Hd, batch=B, c_offset=32400 * C, c_bstride=Nk * C,
                geo=geo, rx=xi, C2=mem, c2_offset=32400 * C, c2_bstride=Nk * C)


def three():
    native.rv_pe_coords(i2l, coords, BV=B * V, h=h, w=w, D=D, pad_h=640.0, pad_w=1600.0, depth_max=54.0,
                        pc_range=pc)
    native.nchw_to_rows(xi, mem, nb=B, nv=V, C=C, HW=h * w, ldy=C, rows_per_batch=Nk, row_offset=32400)
    native.mlp2(coords, W1p, b1, W2p, b2, pos, M=M, K=3 * D, Hd=Hd, R=mem, batch=B, a_bstride=M * 3 * D,
                c_offset=32400 * C, c_bstride=Nk * C, r_offset=32400 * C, r_bstride=Nk * C)


def mlp_only():
    native.mlp2(coords, W1p, b1, W2p, b2, pos, M=M, K=3 * D, Hd=Hd, R=mem, batch=B, a_bstride=M * 3 * D,
                c_offset=32400 * C, c_bstride=Nk * C, r_offset=32400 * C, r_bstride=Nk * C)


def t(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 20 * 1e3


tag = os.environ.get("TAG", "")
print(f"{tag} fused {t(fused):.1f} us | three launches {t(three):.1f} us | one-launch MLP alone {t(mlp_only):.1f} us")
