"""CPU restatement of the CMT / CMTCoop decoder-head forward (PyTorch CPU, fp32).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``projects.mmdet3d_plugin``)
never imports it and has no CPU fallback.

Parity status: **parity unpinned** with respect to reference *outputs*.
The reference (suren3141/CMT-Cooperative-Perception) has no tests, no golden
vectors and no fixtures for this path, and importing or
running it was refused by the environment; that refusal
binds this build.  This restatement is therefore pinned only by
  * closed-form known-answer tests derived by hand from the reference source
    (tests/test_oracle_kat.py), and
  * self-consistency properties (coop with identical agents == single agent,
    final_kernel=1 head == per-query linear, ...).
Every function cites the reference file:line it restates.  Third-party semantics
(mmcv 1.6.2, mmdet 2.28.2, mmdet3d 1.0.0rc6, flash-attn 0.2.2, torch 1.9.1) are
restated from their pinned, published algorithms.

Layouts follow the reference: decoder tensors are sequence-first [N, B, C]
inside the decoder, head outputs are [L, B, Nq, k].
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

__all__ = [
    "inverse_sigmoid", "pos2embed", "coords_bev", "rv_pe", "rv_query_embed",
    "flash_core_fp16", "mha", "decoder", "separate_task_head", "group_layer_norm", "shared_conv",
    "head_forward", "head_coop_forward", "box_epilogue", "decode",
    "denormalize_bbox", "filter_img_metas",
]


# ---------------------------------------------------------------------------
# small math helpers
# ---------------------------------------------------------------------------
def inverse_sigmoid(x, eps=1e-5):
    """mmdet 2.28.2 ``mmdet/models/utils/transformer.py::inverse_sigmoid``
    (imported at reference cmt_head.py:28)."""
    x = x.clamp(min=0, max=1)
    x1 = x.clamp(min=eps)
    x2 = (1 - x).clamp(min=eps)
    return torch.log(x1 / x2)


def pos2embed(pos, num_pos_feats=128, temperature=10000):
    """cmt_head.py:40-50.  NOTE the reference ignores ``temperature``:
    dim_t = 2*(i//2)/F + 1 (quirk reproduced)."""
    scale = 2 * math.pi
    pos = pos * scale
    dim_t = torch.arange(num_pos_feats, dtype=torch.float32)
    dim_t = 2 * torch.div(dim_t, 2, rounding_mode="floor") / num_pos_feats + 1
    pos_x = pos[..., 0, None] / dim_t
    pos_y = pos[..., 1, None] / dim_t
    pos_x = torch.stack((pos_x[..., 0::2].sin(), pos_x[..., 1::2].cos()), dim=-1).flatten(-2)
    pos_y = torch.stack((pos_y[..., 0::2].sin(), pos_y[..., 1::2].cos()), dim=-1).flatten(-2)
    return torch.cat((pos_y, pos_x), dim=-1)


def coords_bev(grid_size, downsample_scale):
    """cmt_head.py:324-337 (x/y naming swap reproduced).  Returns [H*W, 2]."""
    x_size = grid_size[1] // downsample_scale
    y_size = grid_size[0] // downsample_scale
    meshgrid = [[0, x_size - 1, x_size], [0, y_size - 1, y_size]]
    batch_y, batch_x = torch.meshgrid(
        *[torch.linspace(it[0], it[1], it[2]) for it in meshgrid], indexing="ij")
    batch_x = (batch_x + 0.5) / x_size
    batch_y = (batch_y + 0.5) / y_size
    coord_base = torch.cat([batch_x[None], batch_y[None]], dim=0)
    return coord_base.view(2, -1).transpose(1, 0)


def linear(x, w, b=None):
    return F.linear(x, w, b)


def mlp2(x, sd, prefix):
    """nn.Sequential(Linear, ReLU, Linear) -- cmt_head.py:292-301."""
    x = x.to(sd[prefix + ".0.weight"].dtype)
    h = F.relu(linear(x, sd[prefix + ".0.weight"], sd[prefix + ".0.bias"]))
    return linear(h, sd[prefix + ".2.weight"], sd[prefix + ".2.bias"])


def layer_norm(x, w, b, eps=1e-5):
    """mmcv build_norm_layer(dict(type='LN')) == nn.LayerNorm(eps=1e-5)."""
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def _np_inv(m):
    """host fp64 inverse, as np.linalg.inv at cmt_head.py:428,443."""
    return np.linalg.inv(np.asarray(m, dtype=np.float64))


# ---------------------------------------------------------------------------
# coordinate encodings
# ---------------------------------------------------------------------------
def rv_pe(img_hw, img_metas, pc_range, depth_num, sd, prefix="rv_embedding"):
    """cmt_head.py:417-433 (coop: cmt_head_coop.py:283-299).

    img_hw = (H, W) of the image feature map; img_metas[b]['lidar2img'] is a
    list of V 4x4 matrices.  Returns [B*V, H, W, C].  Quirks: pixel top-left
    (arange*pad/H), depth bins use pc_range[3] as max depth."""
    H, W = img_hw
    pad_h, pad_w, _ = img_metas[0]["pad_shape"][0]
    coords_h = torch.arange(H).float() * pad_h / H
    coords_w = torch.arange(W).float() * pad_w / W
    coords_d = 1 + torch.arange(depth_num).float() * (pc_range[3] - 1) / depth_num
    coords_h, coords_w, coords_d = torch.meshgrid([coords_h, coords_w, coords_d], indexing="ij")
    coords = torch.stack([coords_w, coords_h, coords_d, torch.ones_like(coords_h)], dim=-1)
    coords[..., :2] = coords[..., :2] * coords[..., 2:3]
    imgs2lidars = np.concatenate([_np_inv(meta["lidar2img"]) for meta in img_metas])
    imgs2lidars = torch.from_numpy(imgs2lidars).float()
    coords_3d = torch.einsum("hwdo, bco -> bhwdc", coords, imgs2lidars)
    pcr = torch.tensor(pc_range, dtype=torch.float32)
    coords_3d = (coords_3d[..., :3] - pcr[:3]) / (pcr[3:] - pcr[:3])
    return mlp2(coords_3d.reshape(*coords_3d.shape[:-2], -1), sd, prefix)


def rv_query_embed(ref_points, img_metas, pc_range, depth_num, sd, prefix="rv_embedding"):
    """cmt_head.py:439-467 (coop 305-333).  ref_points [B,Nq,3] in [0,1].
    Quirks: z-divide with +-1e-6 sign epsilon (z becomes ~+-1), mask tested
    against pad_shape, masked sum over views."""
    pad_h, pad_w, _ = img_metas[0]["pad_shape"][0]
    dt = ref_points.dtype   # fp32 (eval restatement) or fp64 (training-gradient checks)
    lidars2imgs = torch.from_numpy(np.stack([np.asarray(m["lidar2img"], dtype=np.float64)
                                             for m in img_metas])).float().to(dt)
    imgs2lidars = torch.from_numpy(np.stack([_np_inv(m["lidar2img"]) for m in img_metas])).float().to(dt)
    pcr = torch.tensor(pc_range, dtype=torch.float32).to(dt)
    ref_points = ref_points * (pcr[3:] - pcr[:3]) + pcr[:3]
    proj_points = torch.einsum(
        "bnd, bvcd -> bvnc",
        torch.cat([ref_points, ref_points.new_ones(*ref_points.shape[:-1], 1)], dim=-1),
        lidars2imgs)
    proj = proj_points.clone()
    z_mask = proj[..., 2:3] > 0
    proj[..., :3] = proj_points[..., :3] / (proj_points[..., 2:3] + z_mask * 1e-6 - (~z_mask) * 1e-6)
    mask = (proj[..., 0] < pad_w) & (proj[..., 0] >= 0) & (proj[..., 1] < pad_h) & (proj[..., 1] >= 0)
    mask &= z_mask.squeeze(-1)
    coords_d = (1 + torch.arange(depth_num).float() * (pc_range[3] - 1) / depth_num).to(dt)
    proj = torch.einsum("bvnc, d -> bvndc", proj, coords_d)
    proj = torch.cat([proj[..., :3], proj.new_ones(*proj.shape[:-1], 1)], dim=-1)
    back = torch.einsum("bvndo, bvco -> bvndc", proj, imgs2lidars)
    back = (back[..., :3] - pcr[:3]) / (pcr[3:] - pcr[:3])
    rv = mlp2(back.reshape(*back.shape[:-2], -1), sd, prefix)
    return (rv * mask.unsqueeze(-1)).sum(dim=1)


# ---------------------------------------------------------------------------
# attention / decoder
# ---------------------------------------------------------------------------
def _round_fp16(t):
    return t.to(torch.float16).to(torch.float32)


def flash_core_fp16(q, k, v, scale):
    """The fp16 attention core of flash-attn 0.2.2 as FlashAttention.forward
    calls it (attention.py:46-92): q/k/v rounded to fp16 (auto_fp16), scores and
    row statistics in fp32, P rounded to fp16 before P.V, fp32 accumulation,
    fp16 output (returned here as fp32 values).  q [..., Sq, D], k/v [..., Sk, D]."""
    q, k, v = _round_fp16(q.float()), _round_fp16(k.float()), _round_fp16(v.float())
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    m = s.amax(dim=-1, keepdim=True)
    p = torch.exp(s - m)
    l = p.sum(dim=-1, keepdim=True)
    return _round_fp16(torch.matmul(_round_fp16(p), v) / l)


def mha(query, key, value, in_w, in_b, out_w, out_b, num_heads, core="fp32"):
    """Multi-head attention with a packed in-projection.

    * core='fp32': torch 1.9.1 nn.MultiheadAttention math (self-attn,
      mmcv MultiheadAttention -> F.multi_head_attention_forward).
    * core='fp16': FlashMHA semantics (attention.py:126-138, 46-92):
      projections fp32 (_in_projection_packed, attention.py:21-27), q/k/v
      cast to fp16 by auto_fp16 (attention.py:46), fp32 softmax, P rounded to
      fp16 before P.V (flash-attn 0.2.2 kernel), fp16 output cast back to fp32.
    Inputs/outputs are batch-first [B, S, C]; returns out_proj(context)."""
    wq, wk, wv = in_w.chunk(3)
    bq, bk, bv = in_b.chunk(3) if in_b is not None else (None, None, None)
    q, k, v = linear(query, wq, bq), linear(key, wk, bk), linear(value, wv, bv)
    B, Sq, C = q.shape
    Sk = k.shape[1]
    D = C // num_heads
    q = q.view(B, Sq, num_heads, D).transpose(1, 2)
    k = k.view(B, Sk, num_heads, D).transpose(1, 2)
    v = v.view(B, Sk, num_heads, D).transpose(1, 2)
    scale = 1.0 / math.sqrt(D)
    if core == "fp32":
        s = torch.matmul(q, k.transpose(-1, -2)) * scale
        p = torch.softmax(s, dim=-1)
        o = torch.matmul(p, v)
    elif core == "fp16":
        o = flash_core_fp16(q, k, v, scale)
    else:
        raise ValueError(core)
    o = o.transpose(1, 2).reshape(B, Sq, C)
    return linear(o, out_w, out_b)


def decoder_layer(query, key, query_pos, key_pos, sd, prefix, num_heads, cross_core, self_core):
    """PETRTransformerDecoderLayer (petr_transformer.py:374-487) ->
    mmcv 1.6.2 BaseTransformerLayer.forward with
    operation_order=('self_attn','norm','cross_attn','norm','ffn','norm'),
    post-norm (identity = the pre-attention query), eval mode (no dropout).
    Sequence-first [N, B, C] tensors."""
    # self_attn: mmcv MultiheadAttention: q = k = query+query_pos, v = query
    a = prefix + ".attentions.0.attn."
    q_in = (query + query_pos).transpose(0, 1)
    out = mha(q_in, q_in, query.transpose(0, 1), sd[a + "in_proj_weight"], sd[a + "in_proj_bias"],
              sd[a + "out_proj.weight"], sd[a + "out_proj.bias"], num_heads, self_core)
    query = query + out.transpose(0, 1)
    query = layer_norm(query, sd[prefix + ".norms.0.weight"], sd[prefix + ".norms.0.bias"])
    # cross_attn: PETRMultiheadFlashAttention.forward, petr_transformer.py:282-321
    a = prefix + ".attentions.1.attn."
    q_in = (query + query_pos).transpose(0, 1)
    k_in = (key + key_pos).transpose(0, 1)
    out = mha(q_in, k_in, key.transpose(0, 1), sd[a + "in_proj_weight"], sd[a + "in_proj_bias"],
              sd[a + "out_proj.weight"], sd[a + "out_proj.bias"], num_heads, cross_core)
    query = query + out.transpose(0, 1)
    query = layer_norm(query, sd[prefix + ".norms.1.weight"], sd[prefix + ".norms.1.bias"])
    # ffn: mmcv FFN(num_fcs=2, ReLU, add_identity=True)
    f = prefix + ".ffns.0.layers."
    h = F.relu(linear(query, sd[f + "0.0.weight"], sd[f + "0.0.bias"]))
    query = query + linear(h, sd[f + "1.weight"], sd[f + "1.bias"])
    query = layer_norm(query, sd[prefix + ".norms.2.weight"], sd[prefix + ".norms.2.bias"])
    return query


def decoder(query, memory, query_pos, key_pos, sd, prefix, num_layers, num_heads=8,
            cross_core="fp32", self_core="fp32"):
    """PETRTransformerDecoder.forward, petr_transformer.py:347-371
    (return_intermediate=True, shared post_norm LN on every intermediate; the
    un-normed query feeds the next layer).  Returns [L, Nq, B, C]."""
    inter = []
    for i in range(num_layers):
        query = decoder_layer(query, memory, query_pos, key_pos, sd, f"{prefix}.layers.{i}",
                              num_heads, cross_core, self_core)
        inter.append(layer_norm(query, sd[prefix + ".post_norm.weight"], sd[prefix + ".post_norm.bias"]))
    return torch.stack(inter)


def transformer(bev_mem, img_mem, query_embed, bev_pos, rv_pos, sd, prefix, num_layers,
                num_heads=8, cross_core="fp32", self_core="fp32"):
    """CmtTransformer.forward (cmt_transformer.py:84-127) and its LiDAR
    (166-204) / Image (243-282) variants.
    bev_mem [B,C,H,W] or None; img_mem [B*V,C,h,w] or None; query_embed
    [B,Nq,C]; bev_pos [H*W,C]; rv_pos [B*V,h,w,C].  Returns [L,B,Nq,C]."""
    bs = query_embed.shape[0]
    mems, poss = [], []
    if bev_mem is not None:
        mems.append(bev_mem.flatten(2).permute(2, 0, 1))                      # (h w) bs c
        poss.append(bev_pos.unsqueeze(1).repeat(1, bs, 1))
    if img_mem is not None:
        BV, C, h, w = img_mem.shape
        v = BV // bs
        mems.append(img_mem.view(bs, v, C, h, w).permute(1, 3, 4, 0, 2).reshape(v * h * w, bs, C))
        poss.append(rv_pos.view(bs, v, h, w, C).permute(1, 2, 3, 0, 4).reshape(v * h * w, bs, C))
    memory, pos = torch.cat(mems, 0), torch.cat(poss, 0)
    qpos = query_embed.transpose(0, 1)
    target = torch.zeros_like(qpos)
    out = decoder(target, memory, qpos, pos, sd, prefix + ".decoder", num_layers, num_heads,
                  cross_core, self_core)
    return out.transpose(1, 2)


# ---------------------------------------------------------------------------
# task heads
# ---------------------------------------------------------------------------
def group_layer_norm(x, w, b, groups, eps=1e-6):
    """LayerNormFunction.forward, cmt_head.py:56-66 (biased var, eps 1e-6)."""
    N, C, L = x.shape
    xg = x.view(N, groups, C // groups, L)
    mu = xg.mean(2, keepdim=True)
    var = (xg - mu).pow(2).mean(2, keepdim=True)
    y = (xg - mu) / (var + eps).sqrt()
    return w.view(1, C, 1) * y.view(N, C, L) + b.view(1, C, 1)


def separate_task_head(x, sd, prefix, heads, final_kernel, groups):
    """SeparateTaskHead.forward, cmt_head.py:174-203 (layers built at
    136-162).  x [L,B,Nq,C] -> dict of [L,B,Nq,k].  final_kernel=3 convolves
    along the query axis with zero padding (quirk reproduced)."""
    L, B, Nq, C = x.shape
    xin = x.permute(1, 0, 3, 2).reshape(B, L * C, Nq)       # b (n c) q
    out = {}
    pad = final_kernel // 2
    for head in heads:
        p = f"{prefix}.{head}"
        h = F.conv1d(xin, sd[p + ".0.weight"], None, padding=pad, groups=groups)
        h = group_layer_norm(h, sd[p + ".1.weight"], sd[p + ".1.bias"], groups)
        h = F.relu(h)
        h = F.conv1d(h, sd[p + ".3.weight"], sd[p + ".3.bias"], padding=pad, groups=groups)
        out[head] = h.view(B, L, -1, Nq).permute(1, 0, 3, 2).contiguous()   # n b q c
    return out


def box_epilogue(outs, reference, pc_range):
    """cmt_head.py:501-513: center/height += inverse_sigmoid(ref); sigmoid;
    scale to pc_range.  reference = inverse_sigmoid(ref_points) [B,Nq,3]."""
    center = (outs["center"] + reference[None, :, :, :2]).sigmoid()
    height = (outs["height"] + reference[None, :, :, 2:3]).sigmoid()
    _center, _height = torch.zeros_like(center), torch.zeros_like(height)
    _center[..., 0:1] = center[..., 0:1] * (pc_range[3] - pc_range[0]) + pc_range[0]
    _center[..., 1:2] = center[..., 1:2] * (pc_range[4] - pc_range[1]) + pc_range[1]
    _height[..., 0:1] = height[..., 0:1] * (pc_range[5] - pc_range[2]) + pc_range[2]
    outs["center"] = _center
    outs["height"] = _height
    return outs


def shared_conv(x, sd, prefix="shared_conv"):
    """mmcv ConvModule(Conv2d 3x3 pad 1, no bias, BN2d eval, ReLU) --
    cmt_head.py:280-287, applied at 481."""
    y = F.conv2d(x, sd[prefix + ".conv.weight"], None, padding=1)
    y = F.batch_norm(y, sd[prefix + ".bn.running_mean"], sd[prefix + ".bn.running_var"],
                     sd[prefix + ".bn.weight"], sd[prefix + ".bn.bias"], False, 0.0, 1e-5)
    return F.relu(y)


# ---------------------------------------------------------------------------
# whole head
# ---------------------------------------------------------------------------
def _heads_for(cfg, num_cls):
    heads = dict(cfg["common_heads"])
    heads["cls_logits"] = (num_cls, 2)
    return heads


def _decoder_outputs(cfg, sd, x, x_img, img_metas, ref_points, variant, cross_core, self_core):
    """The per-agent part of forward_single: shared_conv, coordinate
    encodings, transformer, nan_to_num (cmt_head.py:481-499;
    CmtHeadCoop.get_outs_dec cmt_head_coop.py:341-360; LiDAR 1022-1038,
    Image 940-951)."""
    pc_range, depth_num = cfg["pc_range"], cfg["depth_num"]
    C = cfg["hidden_dim"]
    L = cfg["num_layers"]
    if variant != "image":
        x = shared_conv(x, sd)
    bev_pos = rv_pos = None
    if variant != "image":
        cb = coords_bev(cfg["grid_size"], cfg["downsample_scale"])
        bev_pos = mlp2(pos2embed(cb, num_pos_feats=C), sd, "bev_embedding")
    if variant != "lidar":
        rv_pos = rv_pe(x_img.shape[-2:], img_metas, pc_range, depth_num, sd)
    # query_embed: cmt_head.py:469-473 (LiDAR variant 1009-1012)
    rp = inverse_sigmoid(ref_points.clone()).sigmoid()
    q = mlp2(pos2embed(rp, num_pos_feats=C), sd, "bev_embedding")
    if variant != "lidar":
        q = q + rv_query_embed(rp, img_metas, pc_range, depth_num, sd)
    out = transformer(x if variant != "image" else None, x_img if variant != "lidar" else None,
                      q, bev_pos, rv_pos, sd, "transformer", L, cfg["num_heads"],
                      cross_core, self_core)
    return torch.nan_to_num(out)


def _task_outputs(cfg, sd, outs_dec, ref_points, epilogue=True):
    """Task heads; epilogue=False returns the raw logits (center / height
    before + inverse_sigmoid(ref) and sigmoid, cmt_head.py:503-513)."""
    L = cfg["num_layers"]
    reference = inverse_sigmoid(ref_points.clone())
    ret = []
    for t, num_cls in enumerate(cfg["num_classes"]):
        outs = separate_task_head(outs_dec, sd, f"task_heads.{t}", _heads_for(cfg, num_cls),
                                  cfg["final_kernel"], L)
        ret.append(box_epilogue(outs, reference, cfg["pc_range"]) if epilogue else outs)
    return ret


def head_forward(cfg, sd, x, x_img, img_metas, variant="fusion", cross_core="fp32",
                 self_core="fp32", epilogue=True):
    """CmtHead / CmtLidarHead / CmtImageHead ``forward_single`` at eval
    (cmt_head.py:475-547, 1014-1085, 929-999; prepare_for_dn eval branch
    410-413 = repeat of reference_points).  Returns list over tasks of dict
    {center,height,dim,rot,vel,cls_logits} each [L,B,Nq,k]."""
    B = x.shape[0] if x is not None else len(img_metas)
    ref = sd["reference_points.weight"].unsqueeze(0).repeat(B, 1, 1)
    outs_dec = _decoder_outputs(cfg, sd, x, x_img, img_metas, ref, variant, cross_core, self_core)
    return _task_outputs(cfg, sd, outs_dec, ref, epilogue)


def filter_img_metas(img_meta, prefix="", ignore=""):
    """cmt_head_coop.py:41-57."""
    out = {}
    for k, v in img_meta.items():
        if k.startswith(prefix):
            out[k[len(prefix):]] = v
        elif not k.startswith(ignore):
            out[k] = v
    out["node"] = prefix
    return out


def head_coop_forward(cfg, sd, agents, img_metas, variant="fusion", cross_core="fp32",
                      self_core="fp32", epilogue=True):
    """CmtHeadCoop / CmtLidarHeadCoop / CmtImageHeadCoop ``forward_single``
    (cmt_head_coop.py:362-437, 946-1017, 838-911).  ``agents`` is a list of
    (prefix, x, x_img); one decoder pass per agent with shared weights, then an
    element-wise max over agents (388-389; the reference stacks exactly two,
    this restatement folds any number with the same max)."""
    B = len(img_metas)
    ref = sd["reference_points.weight"].unsqueeze(0).repeat(B, 1, 1)
    outs = None
    prefixes = [p for p, _, _ in agents]
    for prefix, x, x_img in agents:
        if variant == "lidar":
            metas = img_metas
        elif set(prefixes) <= {"vehicle_", "infrastructure_"}:
            other = "infrastructure_" if prefix == "vehicle_" else "vehicle_"
            metas = [filter_img_metas(m, prefix, other) for m in img_metas]
        else:   # N agents: drop every other agent's prefixed keys
            metas = [{**{k: v for k, v in m.items() if not any(k.startswith(p) for p in prefixes)},
                      **{k[len(prefix):]: v for k, v in m.items() if k.startswith(prefix)}, "node": prefix}
                     for m in img_metas]
        o = _decoder_outputs(cfg, sd, x, x_img, metas, ref, variant, cross_core, self_core)
        outs = o if outs is None else torch.max(torch.stack([outs, o]), 0).values
    return _task_outputs(cfg, sd, outs, ref, epilogue)


# ---------------------------------------------------------------------------
# box decode
# ---------------------------------------------------------------------------
def denormalize_bbox(nb):
    """core/bbox/util.py:37-68."""
    cx, cy, cz = nb[..., 0:1], nb[..., 1:2], nb[..., 2:3]
    w, l, h = nb[..., 3:4].exp(), nb[..., 4:5].exp(), nb[..., 5:6].exp()
    rot = torch.atan2(nb[..., 6:7], nb[..., 7:8])
    if nb.size(-1) > 8:
        return torch.cat([cx, cy, cz, w, l, h, rot, nb[..., 8:9], nb[..., 9:10]], dim=-1)
    return torch.cat([cx, cy, cz, w, l, h, rot], dim=-1)


def decode(preds, num_classes, max_num, post_center_range, score_threshold=None):
    """MultiTaskBBoxCoder.decode / decode_single
    (multi_task_bbox_coder.py:46-142) followed by the z-shift of get_bboxes
    (cmt_head.py:905-919).  preds: list over tasks of output dicts."""
    bbox_l, logit_l, tid_l = [], [], []
    for t, d in enumerate(preds):
        bbox_l.append(torch.cat((d["center"][-1], d["height"][-1], d["dim"][-1],
                                 d["rot"][-1], d["vel"][-1]), dim=-1))
        logit_l.append(d["cls_logits"][-1])
        tid_l.append(torch.full(d["cls_logits"][-1].shape, t, dtype=torch.int32))
    logits = torch.cat(logit_l, -1)
    bboxes = torch.cat(bbox_l, 1)
    tids = torch.cat(tid_l, -1)
    res = []
    pcr = torch.tensor(post_center_range)
    for i in range(logits.shape[0]):
        cls = logits[i].sigmoid()
        nq = cls.shape[0]
        scores, idx = cls.reshape(-1).topk(max_num)
        labels = idx % num_classes
        bidx = torch.div(idx, num_classes, rounding_mode="floor")
        task = torch.gather(tids[i], 1, labels.unsqueeze(1)).squeeze(1)
        bp = bboxes[i][task * nq + bidx]
        boxes = denormalize_bbox(bp)
        mask = (boxes[..., :3] >= pcr[:3]).all(1) & (boxes[..., :3] <= pcr[3:]).all(1)
        if score_threshold:
            mask &= scores > score_threshold
        boxes = boxes[mask].clone()
        boxes[:, 2] = boxes[:, 2] - boxes[:, 5] * 0.5
        res.append(dict(bboxes=boxes, scores=scores[mask], labels=labels[mask]))
    return res


def cfg_from_head_cfg(head_cfg):
    """Oracle parameters from a reference-style ``pts_bbox_head`` dict."""
    dec = head_cfg["transformer"]["decoder"]
    cfg_pts = head_cfg.get("train_cfg") or head_cfg.get("test_cfg")
    attn = dec["transformerlayers"]["attn_cfgs"][1]
    return dict(
        pc_range=list(head_cfg["bbox_coder"]["pc_range"]),
        depth_num=head_cfg.get("depth_num", 64),
        hidden_dim=head_cfg.get("hidden_dim", 128),
        num_layers=dec["num_layers"],
        num_heads=attn["num_heads"],
        grid_size=cfg_pts["grid_size"],
        downsample_scale=head_cfg.get("downsample_scale", 8),
        common_heads=head_cfg["common_heads"],
        num_classes=[len(t["class_names"]) for t in head_cfg["tasks"]],
        final_kernel=head_cfg["separate_head"]["final_kernel"],
    )
