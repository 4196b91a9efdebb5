"""Closed-form known-answer tests pinning the CPU restatement (oracle/) to the
reference's formulas (SURVEY.md 8(c) KAT list).  The reference ships no test
vectors, so these hand-derived values are the oracle's only external pin."""
import math

import numpy as np
import pytest
import torch

from oracle import cmt_oracle as O


def test_pos2embed_kat():
    """cmt_head.py:40-50, F = 256, (x, y) = (0.4963, 0.7682): output starts
    with the y embedding, dim_t = 1 + 2*(i//2)/F (temperature ignored)."""
    out = O.pos2embed(torch.tensor([[0.4963, 0.7682]]), num_pos_feats=256)[0]
    y = 2 * math.pi * 0.7682
    exp = [math.sin(y), math.cos(y), math.sin(y / 1.0078125), math.cos(y / 1.0078125)]
    assert np.allclose(out[:4].numpy(), exp, atol=1e-5)
    # the values quoted in SURVEY.md 8(a) row a1 (rounded there to ~2e-4)
    assert np.allclose(out[:4].numpy(), [-0.99345, 0.11424, -0.99703, 0.07700], atol=3e-4)
    assert abs(out[256].item() - math.sin(2 * math.pi * 0.4963)) < 1e-5
    assert out.shape == (512,)


def test_coords_bev_kat():
    c = O.coords_bev([1440, 1440, 40], 8)
    assert c.shape == (180 * 180, 2)
    assert torch.allclose(c[0], torch.tensor([0.5 / 180, 0.5 / 180]))
    assert torch.allclose(c[-1], torch.tensor([179.5 / 180, 179.5 / 180]))
    # token t = h*W + w: x follows w, y follows h
    assert torch.allclose(c[1], torch.tensor([1.5 / 180, 0.5 / 180]))
    assert torch.allclose(c[180], torch.tensor([0.5 / 180, 1.5 / 180]))


def test_inverse_sigmoid_kat():
    assert abs(O.inverse_sigmoid(torch.tensor(0.0)).item() - math.log(1e-5)) < 1e-6
    assert abs(O.inverse_sigmoid(torch.tensor(1.0)).item() + math.log(1e-5)) < 1e-6
    x = torch.tensor([0.25, 0.5, 0.9])
    assert torch.allclose(O.inverse_sigmoid(x).sigmoid(), x, atol=1e-6)


def test_group_layer_norm_constant_input_gives_bias():
    N, G, C, L = 2, 3, 64, 5
    x = torch.full((N, G * C, L), 7.0)
    w, b = torch.randn(G * C), torch.randn(G * C)
    y = O.group_layer_norm(x, w, b, G)
    assert torch.allclose(y, b.view(1, -1, 1).expand_as(y), atol=1e-6)


def test_rv_pe_identity_camera():
    """lidar2img = I: token (h, w) at depth d maps to (w*pw/W*d, h*ph/H*d, d),
    normalised by pc_range (cmt_head.py:417-432)."""
    H, W, D = 2, 3, 4
    pc = [-10.0, -10.0, -2.0, 10.0, 10.0, 2.0]
    metas = [{"lidar2img": [np.eye(4)], "pad_shape": [(20, 30, 3)]}]
    captured = {}

    sd = {"rv_embedding.0.weight": torch.eye(12, 3 * D), "rv_embedding.0.bias": torch.zeros(12),
          "rv_embedding.2.weight": torch.eye(12), "rv_embedding.2.bias": torch.zeros(12)}
    # relu(identity MLP) exposes the (non-negative part of the) normalised coordinates
    out = O.rv_pe((H, W), metas, pc, D, sd)
    h, w, k = 1, 2, 3
    d = 1 + k * (pc[3] - 1) / D
    pt = np.array([w * 30 / W * d, h * 20 / H * d, d])
    norm = (pt - np.array(pc[:3])) / (np.array(pc[3:]) - np.array(pc[:3]))
    got = out[0, h, w, 3 * k:3 * k + 3].numpy()
    assert np.allclose(got, np.maximum(norm, 0), atol=1e-5)
    del captured


def _tiny_head_sd(final_kernel=1, L=1, C=256, Nq=8, ncls=3):
    from projects.mmdet3d_plugin import synthetic as S
    cfg, _ = S.make_head_cfg("cmt_lidar_nus", num_query=Nq, num_layers=L, grid_size=[64, 64, 40])
    cfg["separate_head"]["final_kernel"] = final_kernel
    from projects.mmdet3d_plugin import build_head
    torch.manual_seed(0)
    head = build_head(cfg)
    head.init_weights()
    return cfg, S.head_state_dict(head)


def test_task_head_k1_equals_per_query_linear():
    """final_kernel=1 grouped conv == per-query linear per layer group."""
    cfg, sd = _tiny_head_sd(final_kernel=1, L=2)
    heads = dict(cfg["common_heads"], cls_logits=(10, 2))
    x = torch.randn(2, 1, 8, 256)
    out = O.separate_task_head(x, sd, "task_heads.0", heads, 1, 2)
    w1 = sd["task_heads.0.vel.0.weight"][:, :, 0]        # [2*64, 256]
    gw, gb = sd["task_heads.0.vel.1.weight"], sd["task_heads.0.vel.1.bias"]
    w2, b2 = sd["task_heads.0.vel.3.weight"][:, :, 0], sd["task_heads.0.vel.3.bias"]
    for l in range(2):
        h = x[l, 0] @ w1[l * 64:(l + 1) * 64].T
        h = (h - h.mean(1, keepdim=True)) / torch.sqrt(h.var(1, unbiased=False, keepdim=True) + 1e-6)
        h = torch.relu(h * gw[l * 64:(l + 1) * 64] + gb[l * 64:(l + 1) * 64])
        ref = h @ w2[l * 2:(l + 1) * 2].T + b2[l * 2:(l + 1) * 2]
        assert torch.allclose(out["vel"][l, 0], ref, atol=1e-5)


def test_coop_identical_agents_equals_single():
    from projects.mmdet3d_plugin import synthetic as S
    head, cfg, _ = S.build_synthetic_head("cmtcoop_lidar_tumtraf", num_query=16, num_layers=1,
                                          grid_size=[128, 128, 40])
    sd = S.head_state_dict(head)
    oc = O.cfg_from_head_cfg(cfg)
    x = S.synthetic_bev(1, 16, 16, seed=3)
    one = O.head_coop_forward(oc, sd, [("vehicle_", x, None)], [dict()], "lidar")
    two = O.head_coop_forward(oc, sd, [("vehicle_", x, None), ("infrastructure_", x, None)], [dict()], "lidar")
    for k in one[0]:
        assert torch.equal(one[0][k], two[0][k])


def test_filter_img_metas():
    m = {"vehicle_lidar2img": 1, "infrastructure_lidar2img": 2, "sample_idx": 3}
    v = O.filter_img_metas(m, "vehicle_", "infrastructure_")
    assert v == {"lidar2img": 1, "sample_idx": 3, "node": "vehicle_"}


def test_decode_shapes_and_zshift():
    L, B, Nq, ncls = 2, 1, 20, 10
    g = torch.Generator().manual_seed(0)
    d = {"center": torch.rand(L, B, Nq, 2, generator=g) * 10, "height": torch.rand(L, B, Nq, 1, generator=g),
         "dim": torch.randn(L, B, Nq, 3, generator=g) * 0.1, "rot": torch.randn(L, B, Nq, 2, generator=g),
         "vel": torch.randn(L, B, Nq, 2, generator=g), "cls_logits": torch.randn(L, B, Nq, ncls, generator=g)}
    res = O.decode([d], ncls, max_num=15, post_center_range=[-61.2, -61.2, -10, 61.2, 61.2, 10])[0]
    assert res["bboxes"].shape[1] == 9 and res["scores"].shape[0] == res["labels"].shape[0] <= 15
    top = d["cls_logits"][-1, 0].sigmoid().reshape(-1).max()
    assert abs(res["scores"][0].item() - top.item()) < 1e-7


def test_oracle_fp16_core_close_to_fp32():
    """The emulated flash-attn fp16 core stays close to exact attention."""
    g = torch.Generator().manual_seed(1)
    q, k = torch.randn(1, 20, 256, generator=g), torch.randn(1, 300, 256, generator=g)
    w, b = torch.randn(768, 256, generator=g) / 16, torch.randn(768, generator=g)
    ow, ob = torch.randn(256, 256, generator=g) / 16, torch.randn(256, generator=g)
    a = O.mha(q, k, k, w, b, ow, ob, 8, "fp32")
    c = O.mha(q, k, k, w, b, ow, ob, 8, "fp16")
    assert (a - c).abs().max().item() < 5e-3
