"""CPU restatement of the CMT / CMTCoop head TRAINING step (PyTorch CPU,
float64-capable): DN query preparation, the DN self-attention mask, Hungarian
assignment, focal / L1 losses and DN losses.  Gradients come from torch
autograd on this restatement (the reference's own mechanism).

TEST INFRASTRUCTURE ONLY -- imported by tests/ as the checker of the native
training path; never by the product package.  Parity status: unpinned with
respect to reference outputs (no reference fixtures exist and running the
reference was refused); every function cites the reference
file:line or the pinned third-party version it restates.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F
from scipy.optimize import linear_sum_assignment

from . import cmt_oracle as O

__all__ = ["focal_loss", "l1_loss", "focal_cost", "match_cost", "normalize_bbox", "hungarian_assign",
           "prepare_for_dn", "dn_attn_mask", "head_train_forward", "head_loss"]


# ---------------------------------------------------------------------------
# losses (mmdet 2.28.2)
# ---------------------------------------------------------------------------
def focal_loss(logits, labels, label_w, gamma, alpha, loss_weight, avg_factor):
    """mmdet FocalLoss(use_sigmoid=True) -> sigmoid_focal_loss: one-hot targets
    (label == num_classes is background), weights per row, sum / avg_factor."""
    ncls = logits.shape[1]
    t = F.one_hot(labels.long(), ncls + 1)[:, :ncls].to(logits.dtype)
    p = logits.sigmoid()
    pt = (1 - p) * t + p * (1 - t)
    fw = (alpha * t + (1 - alpha) * (1 - t)) * pt.pow(gamma)
    loss = F.binary_cross_entropy_with_logits(logits, t, reduction="none") * fw
    return loss_weight * (loss * label_w[:, None]).sum() / avg_factor


def l1_loss(pred, target, weight, loss_weight, avg_factor):
    """mmdet L1Loss(reduction='mean') with element weights and avg_factor."""
    return loss_weight * ((pred - target).abs() * weight).sum() / avg_factor


def focal_cost(logits, gt_labels, gamma=2.0, alpha=0.25, weight=1.0, eps=1e-12):
    """mmdet FocalLossCost.__call__."""
    p = logits.sigmoid()
    neg = -(1 - p + eps).log() * (1 - alpha) * p.pow(gamma)
    pos = -(p + eps).log() * alpha * (1 - p).pow(gamma)
    return (pos[:, gt_labels] - neg[:, gt_labels]) * weight


def match_cost(logits, boxes, gt_norm, gt_labels, code_w, cls_weight, reg_weight, gamma=2.0, alpha=0.25):
    """HungarianAssigner3D.assign cost (hungarian_assigner_3d.py:120-136) with
    BBox3DL1Cost (match_cost.py:5-27) on the first 8 code-weighted channels."""
    cls = focal_cost(logits, gt_labels.long(), gamma, alpha, cls_weight)
    reg = torch.cdist(boxes[:, :8] * code_w[:8], gt_norm[:, :8] * code_w[:8], p=1) * reg_weight
    return cls + reg


def normalize_bbox(b):
    """core/bbox/util.py:8-34: (cx, cy, cz, log w, log l, log h, sin, cos, vx, vy)."""
    cols = [b[..., 0:3], b[..., 3:6].log(), b[..., 6:7].sin(), b[..., 6:7].cos()]
    if b.shape[-1] > 7:
        cols.append(b[..., 7:9])
    return torch.cat(cols, -1)


def hungarian_assign(cost):
    """scipy linear_sum_assignment on the host (hungarian_assigner_3d.py:139-143):
    (query indices, gt indices)."""
    r, c = linear_sum_assignment(cost.detach().cpu().numpy())
    return torch.from_numpy(r).long(), torch.from_numpy(c).long()


# ---------------------------------------------------------------------------
# DN queries (cmt_head.py:339-415)
# ---------------------------------------------------------------------------
def prepare_for_dn(ref_points, gt_boxes, gt_labels, num_query, scalar, noise_scale, noise_trans, split, pc_range,
                   num_classes, rand_prob):
    """Training branch of prepare_for_dn.  gt_boxes[b] [n_b, 9] with the
    GRAVITY centre (x, y, z_c, w, l, h, yaw, vx, vy); rand_prob [groups * sum n_b, 3]
    is the U(-1, 1) noise the reference draws with torch.rand_like.  Returns
    (padded reference points [B, pad + Nq, 3], pad, single_pad, groups, mask_dict)."""
    B = len(gt_boxes)
    known_num = [t.shape[0] for t in gt_boxes]
    labels = torch.cat(gt_labels)
    boxes = torch.cat(gt_boxes)
    batch_idx = torch.cat([torch.full((n,), i) for i, n in enumerate(known_num)])
    groups = min(scalar, num_query // max(known_num))
    known_indice = torch.arange(labels.numel()).repeat(groups)
    known_labels = labels.repeat(groups).long()
    known_bid = batch_idx.repeat(groups)
    known_bboxs = boxes.repeat(groups, 1)
    center = known_bboxs[:, :3].clone()
    scale = known_bboxs[:, 3:6]
    if noise_scale > 0:
        diff = scale / 2 + noise_trans
        center = center + rand_prob * diff * noise_scale
        pcr = pc_range
        center = torch.stack([(center[:, 0] - pcr[0]) / (pcr[3] - pcr[0]), (center[:, 1] - pcr[1]) / (pcr[4] - pcr[1]),
                              (center[:, 2] - pcr[2]) / (pcr[5] - pcr[2])], -1).clamp(0.0, 1.0)
        mask = torch.norm(rand_prob, 2, 1) > split
        known_labels = known_labels.clone()
        known_labels[mask] = sum(num_classes)
    single_pad = int(max(known_num))
    pad = single_pad * groups
    padded = torch.cat([torch.zeros(pad, 3, dtype=ref_points.dtype), ref_points], 0).unsqueeze(0).repeat(B, 1, 1)
    map_known = torch.cat([torch.arange(n) for n in known_num])
    map_known = torch.cat([map_known + single_pad * i for i in range(groups)]).long()
    padded = padded.index_put((known_bid.long(), map_known), center.to(padded.dtype))
    mask_dict = dict(known_indice=known_indice, batch_idx=batch_idx, map_known_indice=map_known,
                     known_lbs_bboxes=(known_labels, known_bboxs), known_labels_raw=labels.repeat(groups).long(),
                     pad_size=pad)
    return padded, pad, single_pad, groups, mask_dict


def dn_attn_mask(pad, single_pad, groups, num_query):
    """cmt_head.py:386-398 (True = may not attend)."""
    n = pad + num_query
    m = torch.zeros(n, n, dtype=torch.bool)
    m[pad:, :pad] = True
    for i in range(groups):
        lo, hi = single_pad * i, single_pad * (i + 1)
        if i == 0:
            m[lo:hi, hi:pad] = True
        if i == groups - 1:
            m[lo:hi, :lo] = True
        else:
            m[lo:hi, hi:pad] = True
            m[lo:hi, :lo] = True
    return m


# ---------------------------------------------------------------------------
# training forward (eval forward of cmt_oracle + the DN branch)
# ---------------------------------------------------------------------------
def _mha_masked(query, key, value, in_w, in_b, out_w, out_b, num_heads, mask):
    wq, wk, wv = in_w.chunk(3)
    bq, bk, bv = in_b.chunk(3)
    q, k, v = F.linear(query, wq, bq), F.linear(key, wk, bk), F.linear(value, wv, bv)
    B, Sq, C = q.shape
    Sk = k.shape[1]
    D = C // num_heads
    q = q.view(B, Sq, num_heads, D).transpose(1, 2)
    k = k.view(B, Sk, num_heads, D).transpose(1, 2)
    v = v.view(B, Sk, num_heads, D).transpose(1, 2)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    if mask is not None:
        s = s.masked_fill(mask, float("-inf"))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, Sq, C)
    return F.linear(o, out_w, out_b)


def _decoder_train(query, memory, query_pos, key_pos, sd, prefix, L, num_heads, mask):
    """PETRTransformerDecoder with the DN mask on the self-attention
    (attn_masks=[attn_mask, None], cmt_transformer.py:116-121), fp32/fp64 cores."""
    inter = []
    for i in range(L):
        p = f"{prefix}.layers.{i}"
        a = p + ".attentions.0.attn."
        qi = (query + query_pos).transpose(0, 1)
        out = _mha_masked(qi, qi, query.transpose(0, 1), sd[a + "in_proj_weight"], sd[a + "in_proj_bias"],
                          sd[a + "out_proj.weight"], sd[a + "out_proj.bias"], num_heads, mask)
        query = O.layer_norm(query + out.transpose(0, 1), sd[p + ".norms.0.weight"], sd[p + ".norms.0.bias"])
        a = p + ".attentions.1.attn."
        qi = (query + query_pos).transpose(0, 1)
        ki = (memory + key_pos).transpose(0, 1)
        out = _mha_masked(qi, ki, memory.transpose(0, 1), sd[a + "in_proj_weight"], sd[a + "in_proj_bias"],
                          sd[a + "out_proj.weight"], sd[a + "out_proj.bias"], num_heads, None)
        query = O.layer_norm(query + out.transpose(0, 1), sd[p + ".norms.1.weight"], sd[p + ".norms.1.bias"])
        f = p + ".ffns.0.layers."
        h = F.relu(F.linear(query, sd[f + "0.0.weight"], sd[f + "0.0.bias"]))
        query = O.layer_norm(query + F.linear(h, sd[f + "1.weight"], sd[f + "1.bias"]),
                             sd[p + ".norms.2.weight"], sd[p + ".norms.2.bias"])
        inter.append(O.layer_norm(query, sd[prefix + ".post_norm.weight"], sd[prefix + ".post_norm.bias"]))
    return torch.stack(inter)


def _shared_conv_train(x, sd, bn_eps=1e-5):
    """ConvModule in training mode: conv, BatchNorm2d with batch statistics, ReLU."""
    y = F.conv2d(x, sd["shared_conv.conv.weight"], None, padding=1)
    y = F.batch_norm(y, None, None, sd["shared_conv.bn.weight"], sd["shared_conv.bn.bias"], True, 0.0, bn_eps)
    return F.relu(y)


def head_train_forward(cfg, sd, agents, img_metas, variant, ref_padded, pad, single_pad):
    """Training forward of CmtHead / CmtHeadCoop (cmt_head.py:475-547;
    cmt_head_coop.py:362-437) with the padded DN reference points.  ``agents``
    = list of (prefix, x, x_img) (one for CmtHead).  Returns the per-task raw
    output dicts (center / height after the box epilogue) [L, B, pad+Nq, k]."""
    C, L = cfg["hidden_dim"], cfg["num_layers"]
    pc_range, depth_num = cfg["pc_range"], cfg["depth_num"]
    Nq = ref_padded.shape[1] - pad
    mask = dn_attn_mask(pad, single_pad, (pad // single_pad) if single_pad else 0, Nq) if pad else None
    outs = None
    prefixes = [p for p, _, _ in agents]
    for prefix, x, x_img in agents:
        if variant == "lidar" or prefix == "":
            metas = img_metas
        else:
            metas = [{**{k: v for k, v in m.items() if not any(k.startswith(q) for q in prefixes)},
                      **{k[len(prefix):]: v for k, v in m.items() if k.startswith(prefix)}} for m in img_metas]
        mems, poss = [], []
        bs = ref_padded.shape[0]
        if variant != "image":
            xb = _shared_conv_train(x, sd)
            cb = O.coords_bev(cfg["grid_size"], cfg["downsample_scale"]).to(xb.dtype)
            bev_pos = O.mlp2(O.pos2embed(cb, num_pos_feats=C), sd, "bev_embedding")
            mems.append(xb.flatten(2).permute(2, 0, 1))
            poss.append(bev_pos.unsqueeze(1).repeat(1, bs, 1))
        rp = O.inverse_sigmoid(ref_padded.clone()).sigmoid()
        q = O.mlp2(O.pos2embed(rp, num_pos_feats=C), sd, "bev_embedding")
        if variant != "lidar":
            BV, _, h, w = x_img.shape
            v = BV // bs
            rv_pos = O.rv_pe(x_img.shape[-2:], metas, pc_range, depth_num, sd).to(xb.dtype if variant != "image"
                                                                                   else x_img.dtype)
            mems.append(x_img.view(bs, v, C, h, w).permute(1, 3, 4, 0, 2).reshape(v * h * w, bs, C))
            poss.append(rv_pos.view(bs, v, h, w, C).permute(1, 2, 3, 0, 4).reshape(v * h * w, bs, C))
            q = q + O.rv_query_embed(rp, metas, pc_range, depth_num, sd)
        memory, pos = torch.cat(mems, 0), torch.cat(poss, 0)
        qpos = q.transpose(0, 1)
        dec = _decoder_train(torch.zeros_like(qpos), memory, qpos, pos, sd, "transformer.decoder", L,
                             cfg["num_heads"], mask).transpose(1, 2)
        dec = torch.nan_to_num(dec)
        outs = dec if outs is None else torch.max(torch.stack([outs, dec]), 0).values
    return O._task_outputs(cfg, sd, outs, ref_padded)


def _task_targets(pred_boxes, pred_logits, gt_boxes, gt_labels, pc_range, code_w, cls_w, reg_w):
    """_get_targets_single + HungarianAssigner3D for one (sample, task):
    labels [Nq] (ncls = background), label weights (ones), bbox targets [Nq, 9]
    (gravity-centre boxes), bbox weights [Nq, 10], #pos, #neg."""
    Nq, ncls = pred_logits.shape
    labels = torch.full((Nq,), ncls, dtype=torch.long)
    tgt = torch.zeros(Nq, 9, dtype=pred_boxes.dtype)
    bw = torch.zeros(Nq, 10, dtype=pred_boxes.dtype)
    if gt_boxes.shape[0] == 0:
        return labels, torch.ones(Nq, dtype=pred_boxes.dtype), tgt, bw, 0, Nq
    cost = match_cost(pred_logits.detach(), pred_boxes.detach(), normalize_bbox(gt_boxes).to(pred_boxes.dtype),
                      gt_labels, code_w.to(pred_boxes.dtype), cls_w, reg_w)
    r, c = hungarian_assign(cost)
    labels[r] = gt_labels[c].long()
    tgt[r] = gt_boxes[c].to(tgt.dtype)
    bw[r] = 1.0
    return labels, torch.ones(Nq, dtype=pred_boxes.dtype), tgt, bw, r.numel(), Nq - r.numel()


def head_loss(preds, gt_boxes, gt_labels, mask_dict, class_names, pc_range, code_w, loss_cfg, dn_weight, split,
              world_num_tgt=None):
    """CmtHead.loss (cmt_head.py:815-903): per decoder layer loss_single over
    the matching queries and dn_loss_single over the DN queries.  preds: list
    over tasks of dicts with the DN rows in front ([L, B, pad + Nq, k]).
    Returns the reference's loss dict (sum of its values is the training loss)."""
    pad = mask_dict["pad_size"] if mask_dict else 0
    L = preds[0]["center"].shape[0]
    B = preds[0]["center"].shape[1]
    g, a = loss_cfg["gamma"], loss_cfg["alpha"]
    cw_cls, cw_box = loss_cfg["cls_weight"], loss_cfg["box_weight"]
    mw_cls, mw_reg = loss_cfg["match_cls_weight"], loss_cfg["match_reg_weight"]
    losses = {}
    for l in range(L):
        lc_tot = lb_tot = 0.0
        dc_tot = db_tot = 0.0
        flag = 0
        for t, names in enumerate(class_names):
            d = preds[t]
            pb = torch.cat([d[k][l] for k in ("center", "height", "dim", "rot", "vel")], -1)   # [B, pad+Nq, 10]
            pl = d["cls_logits"][l]
            ncls = len(names)
            # ---- matching queries (loss_single / _loss_single_task)
            labs, lws, tgts, bws, npos, nneg = [], [], [], [], 0, 0
            for b in range(B):
                m = (gt_labels[b] >= flag) & (gt_labels[b] < flag + ncls)
                lab, lw, tg, bw, p_, n_ = _task_targets(pb[b, pad:], pl[b, pad:], gt_boxes[b][m],
                                                        gt_labels[b][m] - flag, pc_range, code_w, mw_cls, mw_reg)
                labs.append(lab); lws.append(lw); tgts.append(tg); bws.append(bw)
                npos += p_; nneg += n_
            lab, lw, tg, bw = torch.cat(labs), torch.cat(lws), torch.cat(tgts), torch.cat(bws)
            cls_avg = max(npos * 1.0 + nneg * 0.1, 1)
            lc = focal_loss(pl[:, pad:].reshape(-1, ncls), lab, lw, g, a, cw_cls, cls_avg)
            ntg = normalize_bbox(tg)
            ok = torch.isfinite(ntg).all(-1)
            bwc = bw * code_w.to(bw.dtype)[None]
            lb = l1_loss(pb[:, pad:].reshape(-1, 10)[ok], ntg[ok], bwc[ok], cw_box, npos)
            lc_tot = lc_tot + torch.nan_to_num(lc)
            lb_tot = lb_tot + torch.nan_to_num(lb)
            # ---- DN queries (dn_loss_single / _dn_loss_single_task)
            if pad:
                kl, kb = mask_dict["known_lbs_bboxes"]
                raw = mask_dict["known_labels_raw"]
                new_kl = torch.full_like(kl, ncls)
                new_raw = torch.full_like(raw, ncls)
                for ci in range(ncls):
                    new_kl[kl == ci + flag] = ci
                    new_raw[raw == ci + flag] = ci
                bid = mask_dict["batch_idx"][mask_dict["known_indice"]]
                mk = mask_dict["map_known_indice"]
                dl = pl[bid, mk]
                dbx = pb[bid, mk]
                num_tgt = mask_dict["known_indice"].numel()
                task_mask = new_raw != ncls
                kbx = kb
                if task_mask.sum() > 0:
                    dbx = dbx[task_mask]
                    kbx = kb[task_mask]
                cls_avg_dn = max(num_tgt * 3.14159 / 6 * split * split * split, 1)
                dlc = focal_loss(dl, new_kl, torch.ones(new_kl.shape, dtype=dl.dtype), g, a, cw_cls, cls_avg_dn)
                nt = float(num_tgt) if world_num_tgt is None else world_num_tgt
                nt = max(nt, 1.0)
                nkb = normalize_bbox(kbx)
                ok = torch.isfinite(nkb).all(-1)
                dlb = l1_loss(dbx[ok], nkb[ok].to(dbx.dtype), code_w.to(dbx.dtype)[None].expand(int(ok.sum()), 10),
                              cw_box, nt)
                if task_mask.sum() == 0:
                    dlb = dlb * 0.0
                dc_tot = dc_tot + dn_weight * torch.nan_to_num(dlc)
                db_tot = db_tot + dn_weight * torch.nan_to_num(dlb)
            flag += ncls
        key = "" if l == L - 1 else f"d{l}."
        losses[key + "loss_cls"] = lc_tot
        losses[key + "loss_bbox"] = lb_tot
        if pad:
            losses[key + "dn_loss_cls"] = dc_tot
            losses[key + "dn_loss_bbox"] = db_tot
    return losses
